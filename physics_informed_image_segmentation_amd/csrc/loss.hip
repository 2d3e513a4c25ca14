// Fused segmentation loss for the Stage-II objective (src/loss.py:114-162):
//   0.5 Dice + 0.5 BCE + lambda_RD * mean(r^2) + lambda_PF * mean(eps/2 |grad u|^2 + W(u)/eps)
// with r = D * Lap(u) + u(1-u)(u-a) on reflect-padded 5-point / central
// stencils (src/pde.py:49-212), plus the per-sample thresholded counters the
// step loop turns into Dice and IoU (src/metrics.py:57-71, src/evaluate.py:81-95).
//
// Forward: one pass over p and t (8 B/px from HBM; the stencil neighbours are
// cache hits) -> per-block partial sums -> one finalize block that reduces the
// partials in a fixed order (deterministic) and forms every term.
// Backward: elementwise dL/dp (12 B/px), including the exact adjoint of
// "reflect-pad then stencil": ghost row -1 is row 1 and ghost row n is row
// n-2, so rows 1 and n-2 receive the boundary residual twice.
// No MFMA anywhere: these are bandwidth-bound stencils.
#include "common.h"

namespace pis {

__device__ __forceinline__ int refl(int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }

struct LossArgs {
  const float* p;
  const float* t;
  int B, H, W;
  float dice_w, bce_w, rd_w, pf_w, smooth, D, a, eps, thr;
  int rows_per_block, blocks_per_sample;
  float* fpart;  // [nblk][6]: I, P, T, bce_sum, rd_sum, pf_sum
  int* ipart;    // [nblk][3]: I_hat, P_hat, T_hat
};

template <bool RD, bool PF>
__global__ __launch_bounds__(256) void loss_fwd_kernel(LossArgs g) {
  const int b = blockIdx.y;
  const int y0 = blockIdx.x * g.rows_per_block;
  const int y1 = min(g.H, y0 + g.rows_per_block);
  const int H = g.H, W = g.W;
  const float* u = g.p + (size_t)b * H * W;
  const float* tt = g.t + (size_t)b * H * W;
  float s_it = 0.f, s_p = 0.f, s_t = 0.f, s_bce = 0.f, s_rd = 0.f, s_pf = 0.f;
  int c_i = 0, c_p = 0, c_t = 0;
  const int npx = (y1 - y0) * W;
  for (int k = threadIdx.x; k < npx; k += blockDim.x) {
    const int y = y0 + k / W, x = k % W;
    const float p = u[y * W + x], t = tt[y * W + x];
    s_it = fmaf(p, t, s_it);
    s_p += p;
    s_t += t;
    s_bce += (t - 1.f) * fmaxf(log1pf(-p), -100.f) - t * fmaxf(logf(p), -100.f);
    const bool pb = p > g.thr;
    c_p += pb;
    c_t += t > 0.5f;
    c_i += pb && (t > 0.5f);
    if (RD || PF) {
      const float uu = u[refl(y - 1, H) * W + x], ud = u[refl(y + 1, H) * W + x];
      const float ul = u[y * W + refl(x - 1, W)], ur = u[y * W + refl(x + 1, W)];
      if (RD) {
        const float lap = uu + ud + ul + ur - 4.f * p;
        const float r = g.D * lap + p * (1.f - p) * (p - g.a);
        s_rd = fmaf(r, r, s_rd);
      }
      if (PF) {
        const float gx = 0.5f * (ur - ul), gy = 0.5f * (ud - uu);
        const float q = p * (1.f - p);
        s_pf += 0.5f * g.eps * (gx * gx + gy * gy) + q * q / g.eps;
      }
    }
  }
  float v[6] = {s_it, s_p, s_t, s_bce, s_rd, s_pf};
  int c[3] = {c_i, c_p, c_t};
  __shared__ float fr[4][6];
  __shared__ int ir[4][3];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 6; ++j) v[j] = wave_sum(v[j]);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c[j] += __shfl_xor(c[j], off, 64);
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < 6; ++j) fr[wave][j] = v[j];
#pragma unroll
    for (int j = 0; j < 3; ++j) ir[wave][j] = c[j];
  }
  __syncthreads();
  const int blk = b * g.blocks_per_sample + blockIdx.x;
  if (threadIdx.x < 6)
    g.fpart[blk * 6 + threadIdx.x] = fr[0][threadIdx.x] + fr[1][threadIdx.x] + fr[2][threadIdx.x] + fr[3][threadIdx.x];
  else if (threadIdx.x < 9) {
    const int j = threadIdx.x - 6;
    g.ipart[blk * 3 + j] = ir[0][j] + ir[1][j] + ir[2][j] + ir[3][j];
  }
}

__global__ __launch_bounds__(256) void loss_finalize_kernel(LossArgs g, float* __restrict__ terms,
                                                            int* __restrict__ counts,
                                                            float* __restrict__ scores) {
  const int nblk = g.B * g.blocks_per_sample;
  double s[6] = {0, 0, 0, 0, 0, 0};
  for (int k = threadIdx.x; k < nblk; k += 256)
#pragma unroll
    for (int j = 0; j < 6; ++j) s[j] += (double)g.fpart[k * 6 + j];
  __shared__ double red[4][6];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 6; ++j) s[j] = wave_sum_d(s[j]);
  if (lane == 0)
#pragma unroll
    for (int j = 0; j < 6; ++j) red[wave][j] = s[j];
  __syncthreads();
  if (threadIdx.x == 0) {
    double tot[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) tot[j] = ((red[0][j] + red[1][j]) + red[2][j]) + red[3][j];
    const double n = (double)g.B * g.H * g.W;
    const double I = tot[0], P = tot[1], T = tot[2];
    const double dice = 1.0 - (2.0 * I + g.smooth) / (P + T + g.smooth);
    const double bce = tot[3] / n, rd = tot[4] / n, pf = tot[5] / n;
    double total = g.dice_w * dice + g.bce_w * bce;
    if (g.rd_w > 0.f) total += g.rd_w * rd;
    if (g.pf_w > 0.f) total += g.pf_w * pf;
    terms[0] = (float)total;
    terms[1] = (float)dice;
    terms[2] = (float)bce;
    terms[3] = (float)rd;
    terms[4] = (float)pf;
    terms[5] = (float)I;
    terms[6] = (float)P;
    terms[7] = (float)T;
  }
  for (int b = threadIdx.x; b < g.B; b += 256) {
    long long ci = 0, cp = 0, ct = 0;
    for (int k = 0; k < g.blocks_per_sample; ++k) {
      const int blk = b * g.blocks_per_sample + k;
      ci += g.ipart[blk * 3 + 0];
      cp += g.ipart[blk * 3 + 1];
      ct += g.ipart[blk * 3 + 2];
    }
    if (counts) {
      counts[b * 3 + 0] = (int)ci;
      counts[b * 3 + 1] = (int)cp;
      counts[b * 3 + 2] = (int)ct;
    }
    if (scores) {
      // fp32 arithmetic exactly as the reference metric (src/metrics.py:67-70, evaluate.py:91-94)
      const float fi = (float)ci, fp = (float)cp, ft = (float)ct, sm = g.smooth;
      scores[b * 2 + 0] = (2.f * fi + sm) / (fp + ft + sm);
      scores[b * 2 + 1] = (fi + sm) / (fp + ft - fi + sm);
    }
  }
}

struct LossBwdArgs {
  const float* p;
  const float* t;
  int B, H, W;
  float dice_w, bce_w, rd_w, pf_w, smooth, D, a, eps;
  const float* terms;
  const float* grad_out;
  float* dst;
  int chain;
};

template <bool RD, bool PF>
__global__ __launch_bounds__(256) void loss_bwd_kernel(LossBwdArgs g) {
  const int H = g.H, W = g.W;
  const int64_t HW = (int64_t)H * W, N = (int64_t)g.B * HW;
  const float I = g.terms[5], P = g.terms[6], T = g.terms[7];
  const float S = P + T + g.smooth;
  const float two_i_s = 2.f * I + g.smooth;
  const float inv_s2 = 1.f / (S * S);
  const float go = g.grad_out ? g.grad_out[0] : 1.f;
  const float inv_n = (float)(1.0 / (double)N);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < N;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / HW;
    const int rem = (int)(e - b * HW);
    const int y = rem / W, x = rem - y * W;
    const float* u = g.p + b * HW;
    const float p = u[rem], t = g.t[e];
    float grad = g.dice_w * (-(2.f * t * S - two_i_s) * inv_s2);
    grad += g.bce_w * ((p - t) / fmaxf(p * (1.f - p), 1e-12f) * inv_n);
    if (RD) {
      auto R = [&](int yy, int xx) {
        const float c = u[yy * W + xx];
        const float lap = u[refl(yy - 1, H) * W + xx] + u[refl(yy + 1, H) * W + xx] +
                          u[yy * W + refl(xx - 1, W)] + u[yy * W + refl(xx + 1, W)] - 4.f * c;
        return g.D * lap + c * (1.f - c) * (c - g.a);
      };
      const float rk = R(y, x);
      // adjoint multiplicities of the reflect-padded 5-point stencil
      const int wu = (y >= 1) + (y == 1), wd = (y <= H - 2) + (y == H - 2);
      const int wl = (x >= 1) + (x == 1), wr = (x <= W - 2) + (x == W - 2);
      float adj = -4.f * rk;
      if (wu) adj += wu * R(y - 1, x);
      if (wd) adj += wd * R(y + 1, x);
      if (wl) adj += wl * R(y, x - 1);
      if (wr) adj += wr * R(y, x + 1);
      const float fp = -3.f * p * p + 2.f * (1.f + g.a) * p - g.a;
      grad += g.rd_w * (2.f * inv_n) * (g.D * adj + rk * fp);
    }
    if (PF) {
      auto GX = [&](int yy, int xx) { return 0.5f * (u[yy * W + refl(xx + 1, W)] - u[yy * W + refl(xx - 1, W)]); };
      auto GY = [&](int yy, int xx) { return 0.5f * (u[refl(yy + 1, H) * W + xx] - u[refl(yy - 1, H) * W + xx]); };
      // gx vanishes on columns 0 and W-1 (reflect), so the ghost folds cancel
      float adj = 0.f;
      if (x >= 1) adj += 0.5f * GX(y, x - 1);
      if (x <= W - 2) adj -= 0.5f * GX(y, x + 1);
      if (y >= 1) adj += 0.5f * GY(y - 1, x);
      if (y <= H - 2) adj -= 0.5f * GY(y + 1, x);
      grad += g.pf_w * inv_n * (g.eps * adj + 2.f * p * (1.f - p) * (1.f - 2.f * p) / g.eps);
    }
    grad *= go;
    if (g.chain) grad = grad * (1.f - p) * p;
    g.dst[e] = grad;
  }
}

__global__ void pde_fields_kernel(const float* __restrict__ u0, int B, int H, int W, float D,
                                  float a, float* __restrict__ lap_o, float* __restrict__ res_o,
                                  float* __restrict__ gm_o) {
  const int64_t HW = (int64_t)H * W, N = (int64_t)B * HW;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < N;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / HW;
    const int rem = (int)(e - b * HW), y = rem / W, x = rem - y * W;
    const float* u = u0 + b * HW;
    const float c = u[rem];
    const float uu = u[refl(y - 1, H) * W + x], ud = u[refl(y + 1, H) * W + x];
    const float ul = u[y * W + refl(x - 1, W)], ur = u[y * W + refl(x + 1, W)];
    const float lap = uu + ud + ul + ur - 4.f * c;
    if (lap_o) lap_o[e] = lap;
    if (res_o) res_o[e] = D * lap + c * (1.f - c) * (c - a);
    if (gm_o) {
      const float gx = 0.5f * (ur - ul), gy = 0.5f * (ud - uu);
      gm_o[e] = gx * gx + gy * gy;
    }
  }
}

static void loss_plan(int B, int H, int W, int& rows, int& bps) {
  rows = std::max(1, std::min(H, 4096 / std::max(1, W)));
  bps = (H + rows - 1) / rows;
}

}  // namespace pis

using namespace pis;

extern "C" size_t pis_loss_ws(int B, int H, int W) {
  int rows, bps;
  loss_plan(B, H, W, rows, bps);
  return (size_t)B * bps * (6 * sizeof(float) + 3 * sizeof(int)) + 256;
}

extern "C" int pis_loss_fwd(const float* p, const float* t, int B, int H, int W,
                            const pis_loss_params* prm, float* out_terms, int* counts,
                            float* scores, void* ws, size_t ws_bytes, pis_stream_t stream) {
  PIS_CHECK_ARG(p && t && prm && out_terms && B > 0 && H >= 2 && W >= 2,
                "pis_loss_fwd: bad arguments (reflect padding needs H, W >= 2)");
  PIS_CHECK_ARG(ws && ws_bytes >= pis_loss_ws(B, H, W), "pis_loss_fwd: workspace too small");
  LossArgs g{};
  g.p = p; g.t = t; g.B = B; g.H = H; g.W = W;
  g.dice_w = prm->dice_w; g.bce_w = prm->bce_w; g.rd_w = prm->rd_w; g.pf_w = prm->pf_w;
  g.smooth = prm->smooth; g.D = prm->D; g.a = prm->a; g.eps = prm->eps; g.thr = prm->thr;
  loss_plan(B, H, W, g.rows_per_block, g.blocks_per_sample);
  g.fpart = (float*)ws;
  g.ipart = (int*)((char*)ws + (size_t)B * g.blocks_per_sample * 6 * sizeof(float));
  const bool all = prm->flags & PIS_LOSS_ALL_TERMS;
  const bool rd = all || prm->rd_w > 0.f, pf = all || prm->pf_w > 0.f;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(g.blocks_per_sample, B);
  if (rd && pf) hipLaunchKernelGGL((loss_fwd_kernel<true, true>), grid, dim3(256), 0, s, g);
  else if (rd) hipLaunchKernelGGL((loss_fwd_kernel<true, false>), grid, dim3(256), 0, s, g);
  else if (pf) hipLaunchKernelGGL((loss_fwd_kernel<false, true>), grid, dim3(256), 0, s, g);
  else hipLaunchKernelGGL((loss_fwd_kernel<false, false>), grid, dim3(256), 0, s, g);
  int rc = launch_status("loss_fwd");
  if (rc) return rc;
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, s, g, out_terms, counts, scores);
  return launch_status("loss_finalize");
}

extern "C" int pis_loss_bwd(const float* p, const float* t, int B, int H, int W,
                            const pis_loss_params* prm, const float* terms, const float* grad_out,
                            float* dst, int flags, pis_stream_t stream) {
  PIS_CHECK_ARG(p && t && prm && terms && dst && B > 0 && H >= 2 && W >= 2,
                "pis_loss_bwd: bad arguments");
  LossBwdArgs g{};
  g.p = p; g.t = t; g.B = B; g.H = H; g.W = W;
  g.dice_w = prm->dice_w; g.bce_w = prm->bce_w; g.rd_w = prm->rd_w; g.pf_w = prm->pf_w;
  g.smooth = prm->smooth; g.D = prm->D; g.a = prm->a; g.eps = prm->eps;
  g.terms = terms; g.grad_out = grad_out; g.dst = dst; g.chain = (flags & PIS_LOSS_CHAIN_SIGMOID) ? 1 : 0;
  const int64_t n = (int64_t)B * H * W;
  const int grid = (int)std::min<int64_t>(cdiv(n, 256), 8192);
  hipStream_t s = (hipStream_t)stream;
  const bool rd = prm->rd_w > 0.f, pf = prm->pf_w > 0.f;  // gradient only of terms in the total
  if (rd && pf) hipLaunchKernelGGL((loss_bwd_kernel<true, true>), dim3(grid), dim3(256), 0, s, g);
  else if (rd) hipLaunchKernelGGL((loss_bwd_kernel<true, false>), dim3(grid), dim3(256), 0, s, g);
  else if (pf) hipLaunchKernelGGL((loss_bwd_kernel<false, true>), dim3(grid), dim3(256), 0, s, g);
  else hipLaunchKernelGGL((loss_bwd_kernel<false, false>), dim3(grid), dim3(256), 0, s, g);
  return launch_status("loss_bwd");
}

extern "C" int pis_pde_fields(const float* u, int B, int H, int W, float D, float a, float* lap,
                              float* residual, float* gradmag2, pis_stream_t stream) {
  PIS_CHECK_ARG(u && B > 0 && H >= 2 && W >= 2, "pis_pde_fields: bad arguments");
  const int64_t n = (int64_t)B * H * W;
  const int grid = (int)std::min<int64_t>(cdiv(n, 256), 8192);
  hipLaunchKernelGGL(pde_fields_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, u, B, H, W,
                     D, a, lap, residual, gradmag2);
  return launch_status("pde_fields");
}
