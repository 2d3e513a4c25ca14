// Fused segmentation loss for the Stage-II objective (src/loss.py:114-162):
//   0.5 Dice + 0.5 BCE + lambda_RD * mean(r^2) + lambda_PF * mean(eps/2 |grad u|^2 + W(u)/eps)
// with r = D * Lap(u) + u(1-u)(u-a) on reflect-padded 5-point / central
// stencils (src/pde.py:49-212), plus the per-sample thresholded counters the
// step loop turns into Dice and IoU (src/metrics.py:57-71, src/evaluate.py:81-95).
//
// Forward: one pass over p and t (8 B/px from HBM) in 16x128 pixel tiles, u
// staged in LDS with a 1-pixel reflect halo -> per-tile partial sums -> one
// finalize block that reduces the partials in a fixed order (deterministic).
// Backward: dL/dp (12 B/px) per tile from u staged with a 2-pixel halo and the
// RD residual of the tile (+1 ring) in LDS, including the exact adjoint of
// "reflect-pad then stencil": ghost row -1 is row 1 and ghost row n is row
// n-2, so rows 1 and n-2 receive the boundary residual twice.
// No MFMA anywhere: these are bandwidth-bound stencils.
#include "common.h"

namespace pis {

int reduce_slabs(const float* part, int splits, int64_t n, float* dst, int accumulate, hipStream_t s);

__device__ __forceinline__ int refl(int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }
__device__ __forceinline__ int clampi(int i, int lo, int hi) { return i < lo ? lo : (i > hi ? hi : i); }

// Tiles of LT_Y x LT_X pixels of one sample; u is staged once in LDS with a
// reflect-resolved halo, so every stencil neighbour is an LDS read and HBM sees
// p and t exactly once (rows of the halo are L2 hits of the neighbouring tile).
constexpr int LT_X = 128, LT_Y = 16, LT_S = LT_X + 8;  // LDS row stride; interior at column 4
constexpr int LT_Q = LT_X / 4;                          // float4 chunks per tile row

// s[r * LT_S + 4 + c] = u[refl(y0 - HALO + r)][refl(x0 + c)],  c in [-HALO, LT_X + HALO).
// Full tiles issue every global load of the tile before the first LDS store, so a
// block has its whole footprint in flight at once (these kernels are one wave of
// blocks deep: latency, not issue rate, is what bounds them).
template <int HALO>
__device__ __forceinline__ void stage_tile(const float* __restrict__ u, int H, int W, int y0, int x0,
                                           float* __restrict__ s) {
  constexpr int ROWS = LT_Y + 2 * HALO;
  constexpr int NV = ROWS * LT_Q, NVI = (NV + 255) / 256, NH = ROWS * 2 * HALO;
  static_assert(NH <= 256, "halo columns: one scalar per thread");
  if ((W & 3) == 0 && x0 + LT_X <= W) {
    f32x4 v[NVI];
    float h = 0.f;
#pragma unroll
    for (int j = 0; j < NVI; ++j) {
      const int k = threadIdx.x + 256 * j;
      if (k < NV) {
        const int r = k / LT_Q, q = k % LT_Q;
        const int gy = clampi(refl(y0 - HALO + r, H), 0, H - 1);
        v[j] = *(const f32x4*)(u + (size_t)gy * W + x0 + 4 * q);
      }
    }
    const int hr = threadIdx.x / (2 * HALO), hj = threadIdx.x % (2 * HALO);
    const int hc = hj < HALO ? hj - HALO : LT_X + hj - HALO;
    if (threadIdx.x < NH) {
      const int gy = clampi(refl(y0 - HALO + hr, H), 0, H - 1);
      h = u[(size_t)gy * W + clampi(refl(x0 + hc, W), 0, W - 1)];
    }
#pragma unroll
    for (int j = 0; j < NVI; ++j) {
      const int k = threadIdx.x + 256 * j;
      if (k < NV) *(f32x4*)(s + (k / LT_Q) * LT_S + 4 + 4 * (k % LT_Q)) = v[j];
    }
    if (threadIdx.x < NH) s[hr * LT_S + 4 + hc] = h;
  } else {  // ragged or last tile: element-wise with reflect on both axes
    constexpr int COLS = LT_X + 2 * HALO;
    for (int k = threadIdx.x; k < ROWS * COLS; k += 256) {
      const int r = k / COLS, c = k % COLS - HALO;
      const int gy = clampi(refl(y0 - HALO + r, H), 0, H - 1);
      s[r * LT_S + 4 + c] = u[(size_t)gy * W + clampi(refl(x0 + c, W), 0, W - 1)];
    }
  }
}

// 4 consecutive target values of row y starting at column xb (guarded for ragged W)
__device__ __forceinline__ f32x4 load4(const float* __restrict__ row, int xb, int W) {
  if ((W & 3) == 0) return *(const f32x4*)(row + xb);
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (xb + i < W) v[i] = row[xb + i];
  return v;
}

struct LossArgs {
  const float* p;
  const float* t;
  int B, H, W;
  float dice_w, bce_w, rd_w, pf_w, smooth, D, a, eps, thr;
  float rx;  // 1, or 0 for the diffusion-only residual (PIS_LOSS_NO_REACTION)
  int tiles_x, tiles_y;
  float* fpart;  // [nblk][6]: I, P, T, bce_sum, rd_sum, pf_sum
  int* ipart;    // [nblk][3]: I_hat, P_hat, T_hat
};

template <bool RD, bool PF>
__global__ __launch_bounds__(256) void loss_fwd_kernel(LossArgs g) {
  constexpr bool ST = RD || PF;
  constexpr int HALO = ST ? 1 : 0;
  __shared__ __attribute__((aligned(16))) float su[ST ? (LT_Y + 2) * LT_S : 1];
  const int b = blockIdx.z, y0 = blockIdx.y * LT_Y, x0 = blockIdx.x * LT_X;
  const int H = g.H, W = g.W;
  const float* u = g.p + (size_t)b * H * W;
  const float* tt = g.t + (size_t)b * H * W;
  constexpr int NI = LT_Y * LT_Q / 256;  // 4-pixel items per thread
  f32x4 tvs[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {  // targets in flight together with the tile of u
    const int k = threadIdx.x + 256 * j;
    const int y = y0 + k / LT_Q, xb = x0 + 4 * (k % LT_Q);
    if (y < H && xb < W) tvs[j] = load4(tt + (size_t)y * W, xb, W);
  }
  if constexpr (ST) {
    stage_tile<1>(u, H, W, y0, x0, su);
    __syncthreads();
  }
  // VALU budget is what bounds this kernel (a 4-cycle wave64 VALU op per pixel-term):
  // BCE in log2 units with v_log_f32 (scaled by ln 2 once per thread), the PF
  // terms accumulated unscaled, no divisions.
  constexpr float kLn2 = 0.69314718055994531f, kClamp2 = -144.26950408889634f;  // -100 / ln 2
  float s_it = 0.f, s_p = 0.f, s_t = 0.f, s_bce2 = 0.f, s_rd = 0.f, s_g2 = 0.f, s_q2 = 0.f;
  int c_i = 0, c_p = 0, c_t = 0;
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int k = threadIdx.x + 256 * j;
    const int r = k / LT_Q, q = k % LT_Q;
    const int y = y0 + r, xb = x0 + 4 * q;
    if (y >= H || xb >= W) continue;
    const f32x4 tv = tvs[j];
    f32x4 pv, uv, dv;
    float lft = 0.f, rgt = 0.f;
    if constexpr (ST) {
      const float* sc = su + (r + 1) * LT_S + 4 + 4 * q;
      pv = *(const f32x4*)sc;
      uv = *(const f32x4*)(sc - LT_S);
      dv = *(const f32x4*)(sc + LT_S);
      lft = sc[-1];
      rgt = sc[4];
    } else {
      pv = load4(u + (size_t)y * W, xb, W);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (xb + i >= W) break;
      const float p = pv[i], t = tv[i];
      s_it = fmaf(p, t, s_it);
      s_p += p;
      s_t += t;
      s_bce2 += (t - 1.f) * fmaxf(__builtin_amdgcn_logf(1.f - p), kClamp2) -
                t * fmaxf(__builtin_amdgcn_logf(p), kClamp2);
      const bool pb = p > g.thr, tb = t > 0.5f;
      c_p += pb;
      c_t += tb;
      c_i += pb && tb;
      if constexpr (ST) {
        const float ul = i == 0 ? lft : pv[i - 1], ur = i == 3 ? rgt : pv[i + 1];
        const float uu = uv[i], ud = dv[i];
        const float qq = fmaf(-p, p, p);  // p (1 - p)
        if (RD) {
          const float lap = (uu + ud) + (ul + ur) - 4.f * p;
          const float rr = fmaf(g.D, lap, g.rx * qq * (p - g.a));
          s_rd = fmaf(rr, rr, s_rd);
        }
        if (PF) {
          const float gx = ur - ul, gy = ud - uu;  // 2x the central differences
          s_g2 = fmaf(gx, gx, fmaf(gy, gy, s_g2));
          s_q2 = fmaf(qq, qq, s_q2);
        }
      }
    }
  }
  const float s_bce = s_bce2 * kLn2;
  const float s_pf = 0.125f * g.eps * s_g2 + s_q2 / g.eps;
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
  const int blk = (b * g.tiles_y + blockIdx.y) * g.tiles_x + blockIdx.x;
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
  const int bps = g.tiles_x * g.tiles_y;
  const int nblk = g.B * bps;
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
  // per-sample counters: one wave per sample, lanes stride over the sample's tiles
  for (int b = wave; b < g.B; b += 4) {
    long long ci = 0, cp = 0, ct = 0;
    for (int k = lane; k < bps; k += 64) {
      const int blk = b * bps + k;
      ci += g.ipart[blk * 3 + 0];
      cp += g.ipart[blk * 3 + 1];
      ct += g.ipart[blk * 3 + 2];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      ci += __shfl_xor(ci, off, 64);
      cp += __shfl_xor(cp, off, 64);
      ct += __shfl_xor(ct, off, 64);
    }
    if (lane == 0) {
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
}

// ---------------------------------------------------------------------------
// Forward for W % 4 == 0 (the training shapes): a block owns `rows` whole image rows of one
// sample (~4096 px); each thread streams float4 items with all loads of four items in flight
// before their arithmetic (no LDS staging, no barrier): the up/down neighbour rows and the
// left/right ghosts (reflect: column -1 is column 1, W is W-2) are re-reads of lines the block
// itself fetches, served by L1/L2, so HBM sees p and t about once. A one-block finalize launch
// reduces the per-block partials in a fixed order (double, four partials in flight per
// thread, fixed butterflies): deterministic.
// ---------------------------------------------------------------------------
struct LossRowArgs {
  LossArgs g;
  int rows;             // image rows per block
  int bands;            // blocks per sample
  float* terms;
  int* counts;
  float* scores;
};

template <bool RD, bool PF>
__global__ __launch_bounds__(256) void loss_fwd_rows_kernel(LossRowArgs a) {
  constexpr bool ST = RD || PF;
  const LossArgs& g = a.g;
  const int H = g.H, W = g.W, W4 = W >> 2;
  const int band = blockIdx.x, b = blockIdx.y;
  const int y0 = band * a.rows, nr = min(a.rows, H - y0);
  const float* u = g.p + (size_t)b * H * W;
  const float* tt = g.t + (size_t)b * H * W;
  const int items = nr * W4;  // float4 items of the block's rows
  constexpr float kLn2 = 0.69314718055994531f, kClamp2 = -144.26950408889634f;  // -100 / ln 2
  float s_it = 0.f, s_p = 0.f, s_t = 0.f, s_bce2 = 0.f, s_rd = 0.f, s_g2 = 0.f, s_q2 = 0.f;
  int c_i = 0, c_p = 0, c_t = 0;
  constexpr int U = 4;  // items per thread in flight
  for (int k0 = threadIdx.x; k0 < items; k0 += U * 256) {
    f32x4 tv[U], pv[U], uv[U], dv[U];
    float lft[U], rgt[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {  // every load of U items first, then the arithmetic
      const int k = min(k0 + 256 * j, items - 1);  // tail items recompute the last one, discarded below
      const int r = k / W4, xb = 4 * (k - r * W4), y = y0 + r;
      const float* row = u + (size_t)y * W;
      tv[j] = *(const f32x4*)(tt + (size_t)y * W + xb);
      pv[j] = *(const f32x4*)(row + xb);
      if constexpr (ST) {
        uv[j] = *(const f32x4*)(u + (size_t)refl(y - 1, H) * W + xb);  // reflect: row -1 is row 1
        dv[j] = *(const f32x4*)(u + (size_t)refl(y + 1, H) * W + xb);  // row H is row H-2
        lft[j] = row[xb == 0 ? 1 : xb - 1];                             // column -1 is column 1
        rgt[j] = row[xb + 4 == W ? W - 2 : xb + 4];                     // column W is column W-2
      }
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (k0 + 256 * j >= items) break;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = pv[j][i], t = tv[j][i];
        s_it = fmaf(p, t, s_it);
        s_p += p;
        s_t += t;
        s_bce2 += (t - 1.f) * fmaxf(__builtin_amdgcn_logf(1.f - p), kClamp2) -
                  t * fmaxf(__builtin_amdgcn_logf(p), kClamp2);
        const bool pb = p > g.thr, tb = t > 0.5f;
        c_p += pb;
        c_t += tb;
        c_i += pb && tb;
        if constexpr (ST) {
          const float ul = i == 0 ? lft[j] : pv[j][i - 1], ur = i == 3 ? rgt[j] : pv[j][i + 1];
          const float uu = uv[j][i], ud = dv[j][i];
          const float qq = fmaf(-p, p, p);  // p (1 - p)
          if (RD) {
            const float lap = (uu + ud) + (ul + ur) - 4.f * p;
            const float rr = fmaf(g.D, lap, g.rx * qq * (p - g.a));
            s_rd = fmaf(rr, rr, s_rd);
          }
          if (PF) {
            const float gx = ur - ul, gy = ud - uu;  // 2x the central differences
            s_g2 = fmaf(gx, gx, fmaf(gy, gy, s_g2));
            s_q2 = fmaf(qq, qq, s_q2);
          }
        }
      }
    }
  }
  float v[6] = {s_it, s_p, s_t, s_bce2 * kLn2, s_rd, 0.125f * g.eps * s_g2 + s_q2 / g.eps};
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
  const int blk = b * a.bands + band;
  if (threadIdx.x < 6) {
    g.fpart[blk * 6 + threadIdx.x] = ((fr[0][threadIdx.x] + fr[1][threadIdx.x]) + fr[2][threadIdx.x]) + fr[3][threadIdx.x];
  } else if (threadIdx.x < 9) {
    const int j = threadIdx.x - 6;
    g.ipart[blk * 3 + j] = ir[0][j] + ir[1][j] + ir[2][j] + ir[3][j];
  }
}

// The fixed-order reduction of the row kernel's partials (one block of 1024 threads; the launch
// boundary is the hand-off — an in-kernel last-arriver hand-off costs an agent-scope L2 write-back
// per block, measured 2x slower at C2). Every partial is first copied to LDS with all loads in
// flight (one memory round trip), then reduced from LDS: thread k sums blocks k, k + 1024, ... in
// double, fixed butterflies; per-sample counters one wave per sample.
constexpr int LOSS_MAX_BLOCKS = 2048;

__global__ __launch_bounds__(1024) void loss_finalize_rows_kernel(LossRowArgs a) {
  __shared__ float sf[LOSS_MAX_BLOCKS * 6];
  __shared__ int si[LOSS_MAX_BLOCKS * 3];
  const LossArgs& g = a.g;
  const int nblk = g.B * a.bands, bps = a.bands;
  for (int k = threadIdx.x; k < nblk * 6; k += 1024) sf[k] = g.fpart[k];
  for (int k = threadIdx.x; k < nblk * 3; k += 1024) si[k] = g.ipart[k];
  __syncthreads();
  double s[6] = {0, 0, 0, 0, 0, 0};
  for (int k = threadIdx.x; k < nblk; k += 1024)
#pragma unroll
    for (int j = 0; j < 6; ++j) s[j] += (double)sf[k * 6 + j];
  __shared__ double red[16][6];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 6; ++j) s[j] = wave_sum_d(s[j]);
  if (lane == 0)
#pragma unroll
    for (int j = 0; j < 6; ++j) red[wave][j] = s[j];
  for (int b = wave; b < g.B; b += 16) {
    long long ci = 0, cp = 0, ct = 0;
    for (int k = lane; k < bps; k += 64) {
      const int blk = b * bps + k;
      ci += si[blk * 3 + 0];
      cp += si[blk * 3 + 1];
      ct += si[blk * 3 + 2];
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      ci += __shfl_xor(ci, off, 64);
      cp += __shfl_xor(cp, off, 64);
      ct += __shfl_xor(ct, off, 64);
    }
    if (lane == 0) {
      if (a.counts) {
        a.counts[b * 3 + 0] = (int)ci;
        a.counts[b * 3 + 1] = (int)cp;
        a.counts[b * 3 + 2] = (int)ct;
      }
      if (a.scores) {  // fp32 arithmetic exactly as the reference metric (src/metrics.py:67-70, evaluate.py:91-94)
        const float fi = (float)ci, fp = (float)cp, ft = (float)ct, sm = g.smooth;
        a.scores[b * 2 + 0] = (2.f * fi + sm) / (fp + ft + sm);
        a.scores[b * 2 + 1] = (fi + sm) / (fp + ft - fi + sm);
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double tot[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      tot[j] = red[0][j];
      for (int w = 1; w < 16; ++w) tot[j] += red[w][j];
    }
    const double n = (double)g.B * g.H * g.W;
    const double I = tot[0], P = tot[1], T = tot[2];
    const double dice = 1.0 - (2.0 * I + g.smooth) / (P + T + g.smooth);
    const double bce = tot[3] / n, rd = tot[4] / n, pf = tot[5] / n;
    double total = g.dice_w * dice + g.bce_w * bce;
    if (g.rd_w > 0.f) total += g.rd_w * rd;
    if (g.pf_w > 0.f) total += g.pf_w * pf;
    float* terms = a.terms;
    terms[0] = (float)total;
    terms[1] = (float)dice;
    terms[2] = (float)bce;
    terms[3] = (float)rd;
    terms[4] = (float)pf;
    terms[5] = (float)I;
    terms[6] = (float)P;
    terms[7] = (float)T;
  }
}

// rows per block of the whole-row forward: at least ~4096 pixels (4 float4 items per thread), and
// few enough blocks that the finalize stages every partial in LDS (<= LOSS_MAX_BLOCKS)
static int loss_rows(int B, int H, int W) {
  int r = std::max(1, 4096 / W);
  while ((int64_t)B * cdiv(H, r) > LOSS_MAX_BLOCKS) r *= 2;
  return std::min(r, H);
}
static bool loss_rows_ok(int B, int H, int W) {
  return (W & 3) == 0 && H >= 2 && W >= 8 && B <= LOSS_MAX_BLOCKS;
}

struct LossBwdArgs {
  const float* p;
  const float* t;
  int B, H, W;
  float dice_w, bce_w, rd_w, pf_w, smooth, D, a, eps;
  float rx;  // 1, or 0 for the diffusion-only residual (PIS_LOSS_NO_REACTION)
  const float* terms;
  const float* grad_out;
  float* dst;
  int chain;
};

template <bool RD, bool PF>
__global__ __launch_bounds__(256) void loss_bwd_kernel(LossBwdArgs g) {
  constexpr bool ST = RD || PF;
  __shared__ __attribute__((aligned(16))) float su[ST ? (LT_Y + 4) * LT_S : 1];
  __shared__ __attribute__((aligned(16))) float sr[RD ? (LT_Y + 2) * LT_S : 1];
  const int b = blockIdx.z, y0 = blockIdx.y * LT_Y, x0 = blockIdx.x * LT_X;
  const int H = g.H, W = g.W;
  const size_t HW = (size_t)H * W;
  const float* u = g.p + b * HW;
  const float* tt = g.t + b * HW;
  float* dd = g.dst + b * HW;
  // block-uniform coefficients; dL/dp = cA + cT t + BCE + RD + PF, no divisions per pixel
  const float I = g.terms[5], P = g.terms[6], T = g.terms[7];
  const float S = P + T + g.smooth;
  const float go = g.grad_out ? g.grad_out[0] : 1.f;
  const float inv_n = (float)(1.0 / ((double)g.B * HW));
  const float inv_s2 = 1.f / (S * S);
  const float cA = go * g.dice_w * (2.f * I + g.smooth) * inv_s2;
  const float cT = -go * g.dice_w * 2.f * S * inv_s2;
  const float cB = go * g.bce_w * inv_n;
  const float cR = go * g.rd_w * 2.f * inv_n, cRD = cR * g.D;
  const float cPa = go * g.pf_w * inv_n * g.eps * 0.25f, cPw = go * g.pf_w * inv_n * 2.f / g.eps;
  const float fa = 2.f * (1.f + g.a);
  constexpr int NI = LT_Y * LT_Q / 256;  // 4-pixel items per thread
  f32x4 tvs[NI];
#pragma unroll
  for (int j = 0; j < NI; ++j) {  // targets in flight together with the tile of u
    const int k = threadIdx.x + 256 * j;
    const int y = y0 + k / LT_Q, xb = x0 + 4 * (k % LT_Q);
    if (y < H && xb < W) tvs[j] = load4(tt + (size_t)y * W, xb, W);
  }
  if constexpr (ST) {
    stage_tile<2>(u, H, W, y0, x0, su);
    __syncthreads();
  }
  if constexpr (RD) {
    // residual r = D Lap(u) + u(1-u)(u-a) on rows y0-1 .. y0+LT_Y, columns x0-1 .. x0+LT_X
    // (zero outside the image: those slots only meet zero adjoint weights)
    constexpr int NR = (LT_Y + 2) * LT_Q;
    for (int k = threadIdx.x; k < NR + (LT_Y + 2) * 2; k += 256) {
      if (k < NR) {  // 4 interior columns
        const int rr = k / LT_Q, q = k % LT_Q;
        const int yy = y0 - 1 + rr;
        const float* sc = su + (rr + 1) * LT_S + 4 + 4 * q;
        const f32x4 c = *(const f32x4*)sc, up = *(const f32x4*)(sc - LT_S), dn = *(const f32x4*)(sc + LT_S);
        const float lft = sc[-1], rgt = sc[4];
        f32x4 out;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float c0 = c[i];
          const float ul = i == 0 ? lft : c[i - 1], ur = i == 3 ? rgt : c[i + 1];
          const float lap = (up[i] + dn[i]) + (ul + ur) - 4.f * c0;
          const bool ok = yy >= 0 && yy < H && x0 + 4 * q + i < W;
          out[i] = ok ? fmaf(g.D, lap, g.rx * fmaf(-c0, c0, c0) * (c0 - g.a)) : 0.f;
        }
        *(f32x4*)(sr + rr * LT_S + 4 + 4 * q) = out;
      } else {  // edge columns x0-1 and x0+LT_X
        const int e = k - NR, rr = e >> 1, cc = (e & 1) ? LT_X : -1;
        const int yy = y0 - 1 + rr, xx = x0 + cc;
        float r = 0.f;
        if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
          const float* sc = su + (rr + 1) * LT_S + 4 + cc;
          const float c0 = sc[0];
          const float lap = (sc[-LT_S] + sc[LT_S]) + (sc[-1] + sc[1]) - 4.f * c0;
          r = fmaf(g.D, lap, g.rx * fmaf(-c0, c0, c0) * (c0 - g.a));
        }
        sr[rr * LT_S + 4 + cc] = r;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < NI; ++j) {
    const int k = threadIdx.x + 256 * j;
    const int r = k / LT_Q, q = k % LT_Q;
    const int y = y0 + r, xb = x0 + 4 * q;
    if (y >= H || xb >= W) continue;
    const f32x4 tv = tvs[j];
    const float* sc = su + (r + 2) * LT_S + 4 + 4 * q;
    const f32x4 pv = ST ? *(const f32x4*)sc : load4(u + (size_t)y * W, xb, W);
    f32x4 rc, ru, rd;
    float rl = 0.f, rrt = 0.f;
    if constexpr (RD) {
      const float* sq = sr + (r + 1) * LT_S + 4 + 4 * q;
      rc = *(const f32x4*)sq;
      ru = *(const f32x4*)(sq - LT_S);
      rd = *(const f32x4*)(sq + LT_S);
      rl = sq[-1];
      rrt = sq[4];
    }
    f32x4 u2, d2;
    float l2[2] = {0.f, 0.f}, r2[2] = {0.f, 0.f};
    if constexpr (PF) {
      u2 = *(const f32x4*)(sc - 2 * LT_S);
      d2 = *(const f32x4*)(sc + 2 * LT_S);
      l2[0] = sc[-2];
      l2[1] = sc[-1];
      r2[0] = sc[4];
      r2[1] = sc[5];
    }
    f32x4 out;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int x = xb + i;
      const float p = pv[i], t = tv[i];
      const float qq = fmaf(-p, p, p);  // p (1 - p)
      float grad = fmaf(cT, t, cA);
      grad = fmaf(cB * (p - t), __builtin_amdgcn_rcpf(fmaxf(qq, 1e-12f)), grad);
      if constexpr (RD) {
        // adjoint of the reflect-padded 5-point stencil: ghost row -1 is row 1 and ghost
        // row H is row H-2, so rows/columns 1 and n-2 receive the boundary residual twice
        const float rk = rc[i];
        const float rl_ = i == 0 ? rl : rc[i - 1], rr_ = i == 3 ? rrt : rc[i + 1];
        float adj = (ru[i] + rd[i]) + (rl_ + rr_) - 4.f * rk;
        adj += (y == 1 ? ru[i] : 0.f) + (y == H - 2 ? rd[i] : 0.f);
        adj += (x == 1 ? rl_ : 0.f) + (x == W - 2 ? rr_ : 0.f);
        const float fp = g.rx * fmaf(p, fmaf(-3.f, p, fa), -g.a);
        grad = fmaf(cRD, adj, fmaf(cR * rk, fp, grad));
      }
      if constexpr (PF) {
        // gx vanishes on columns 0 and W-1 (reflect), so the ghost folds cancel
        const float xm2 = i < 2 ? l2[i] : pv[i - 2], xp2 = i >= 2 ? r2[i - 2] : pv[i + 2];
        float adj = 0.f;
        adj += x >= 1 ? p - xm2 : 0.f;
        adj -= x <= W - 2 ? xp2 - p : 0.f;
        adj += y >= 1 ? p - u2[i] : 0.f;
        adj -= y <= H - 2 ? d2[i] - p : 0.f;
        grad = fmaf(cPa, adj, fmaf(cPw * qq, 1.f - 2.f * p, grad));
      }
      if (g.chain) grad *= qq;
      out[i] = grad;
    }
    if ((W & 3) == 0) {
      *(f32x4*)(dd + (size_t)y * W + xb) = out;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (xb + i < W) dd[(size_t)y * W + xb + i] = out[i];
    }
  }
}

// ---------------------------------------------------------------------------
// Loss backward fused into the head backward (the consumer of dL/du): one
// block = R whole image rows. The block stages u for rows y0-2 .. y0+R+1 (reflect
// resolved, 2 halo columns), the RD residual of rows y0-1 .. y0+R, and dL/dz of
// its R*W pixels in LDS, then streams the 64-channel head input exactly like
// head_bwd_kernel: dx = dz w (x > 0), dw/db partial sums per block. dL/dz never
// goes to HBM and the loss costs no launch of its own.
// ---------------------------------------------------------------------------
struct HeadLossArgs {
  const float* x; int ldx;
  const float* w;
  const float* u;
  const float* t;
  float* du_out;          // optional: dL/du (before the sigmoid chain) for autograd
  int B, H, W, C, R;
  float dice_w, bce_w, rd_w, pf_w, smooth, D, a, eps;
  float rx;  // 1, or 0 for the diffusion-only residual (PIS_LOSS_NO_REACTION)
  const float* terms;
  const float* grad_out;
  float* dx; int lddx;
  float* part;    // [blocks][C]
  float* part_b;  // [blocks]
};

template <bool RD, bool PF>
__global__ __launch_bounds__(256) void head_loss_bwd_kernel(HeadLossArgs g) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int H = g.H, W = g.W, SW = W + 4, SR = W + 2;
  const int b = blockIdx.y, y0 = blockIdx.x * g.R, nr = min(g.R, H - y0);
  float* su = smem;                                     // [(R+4)][SW], column c at c + 2
  float* sr = su + (g.R + 4) * SW;                      // [(R+2)][SR], column c at c + 1
  float* sdz = sr + (RD ? (g.R + 2) * SR : 0);          // [R][W]
  const size_t HW = (size_t)H * W;
  const float* u = g.u + b * HW;
  const float* tt = g.t + b * HW;

  const float I = g.terms[5], P = g.terms[6], T = g.terms[7];
  const float S = P + T + g.smooth;
  const float go = g.grad_out ? g.grad_out[0] : 1.f;
  const float inv_n = (float)(1.0 / ((double)g.B * HW));
  const float inv_s2 = 1.f / (S * S);
  const float cA = go * g.dice_w * (2.f * I + g.smooth) * inv_s2;
  const float cT = -go * g.dice_w * 2.f * S * inv_s2;
  const float cB = go * g.bce_w * inv_n;
  const float cR = go * g.rd_w * 2.f * inv_n, cRD = cR * g.D;
  const float cPa = go * g.pf_w * inv_n * g.eps * 0.25f, cPw = go * g.pf_w * inv_n * 2.f / g.eps;
  const float fa = 2.f * (1.f + g.a);

  for (int k = threadIdx.x; k < (nr + 4) * SW; k += 256) {
    const int r = k / SW, c = k - r * SW - 2;
    const int gy = clampi(refl(y0 - 2 + r, H), 0, H - 1), gx = clampi(refl(c, W), 0, W - 1);
    su[k] = u[(size_t)gy * W + gx];
  }
  __syncthreads();
  if constexpr (RD) {
    for (int k = threadIdx.x; k < (nr + 2) * SR; k += 256) {
      const int rr = k / SR, cc = k - rr * SR - 1;
      const int yy = y0 - 1 + rr;
      float r = 0.f;
      if (yy >= 0 && yy < H && cc >= 0 && cc < W) {
        const float* sc = su + (rr + 1) * SW + cc + 2;
        const float c0 = sc[0];
        const float lap = (sc[-SW] + sc[SW]) + (sc[-1] + sc[1]) - 4.f * c0;
        r = fmaf(g.D, lap, g.rx * fmaf(-c0, c0, c0) * (c0 - g.a));
      }
      sr[k] = r;
    }
    __syncthreads();
  }
  for (int k = threadIdx.x; k < nr * W; k += 256) {
    const int r = k / W, x = k - r * W, y = y0 + r;
    const float* sc = su + (r + 2) * SW + x + 2;
    const float p = sc[0], t = tt[(size_t)y * W + x];
    const float qq = fmaf(-p, p, p);
    float grad = fmaf(cT, t, cA);
    grad = fmaf(cB * (p - t), __builtin_amdgcn_rcpf(fmaxf(qq, 1e-12f)), grad);
    if constexpr (RD) {
      const float* sq = sr + (r + 1) * SR + x + 1;
      const float rk = sq[0], ru = sq[-SR], rd = sq[SR], rl = sq[-1], rrt = sq[1];
      float adj = (ru + rd) + (rl + rrt) - 4.f * rk;
      adj += (y == 1 ? ru : 0.f) + (y == H - 2 ? rd : 0.f);
      adj += (x == 1 ? rl : 0.f) + (x == W - 2 ? rrt : 0.f);
      const float fp = g.rx * fmaf(p, fmaf(-3.f, p, fa), -g.a);
      grad = fmaf(cRD, adj, fmaf(cR * rk, fp, grad));
    }
    if constexpr (PF) {
      float adj = 0.f;
      adj += x >= 1 ? p - sc[-2] : 0.f;
      adj -= x <= W - 2 ? sc[2] - p : 0.f;
      adj += y >= 1 ? p - sc[-2 * SW] : 0.f;
      adj -= y <= H - 2 ? sc[2 * SW] - p : 0.f;
      grad = fmaf(cPa, adj, fmaf(cPw * qq, 1.f - 2.f * p, grad));
    }
    if (g.du_out) g.du_out[b * HW + (size_t)y * W + x] = grad;
    sdz[k] = grad * qq;  // sigmoid chain: dz = dL/du * u (1 - u)
  }
  __syncthreads();

  // head backward over the block's pixels (C/4 lanes per pixel, as head_bwd_kernel)
  const int c4n = g.C / 4, rows = 256 / c4n;
  const int pr = threadIdx.x / c4n, c4 = threadIdx.x - pr * c4n;
  const int64_t p0 = (int64_t)b * HW + (int64_t)y0 * W;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float accb = 0.f;
  if (pr < rows) {
    const f32x4 wv = *reinterpret_cast<const f32x4*>(g.w + 4 * c4);
    for (int k = pr; k < nr * W; k += rows) {
      const float d = sdz[k];
      if (c4 == 0) accb += d;
      const int64_t pix = p0 + k;
      const f32x4 xv = *reinterpret_cast<const f32x4*>(g.x + pix * g.ldx + 4 * c4);
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = xv[j] > 0.f ? d * wv[j] : 0.f;
        acc[j] = fmaf(d, xv[j], acc[j]);
      }
      *reinterpret_cast<f32x4*>(g.dx + pix * g.lddx + 4 * c4) = o;
    }
  }
  __syncthreads();  // sdz is dead: reuse the staging area for the block reduction
  f32x4* red = reinterpret_cast<f32x4*>(smem);
  float* redb = reinterpret_cast<float*>(red + 256);
  red[threadIdx.x] = acc;
  redb[threadIdx.x] = accb;
  __syncthreads();
  const int blk = blockIdx.y * gridDim.x + blockIdx.x;
  if ((int)threadIdx.x < c4n) {
    f32x4 s4 = red[threadIdx.x];
    for (int k = 1; k < rows; ++k) s4 += red[k * c4n + threadIdx.x];
    *reinterpret_cast<f32x4*>(g.part + (size_t)blk * g.C + 4 * threadIdx.x) = s4;
  }
  if (threadIdx.x == 0) {
    float s1 = 0.f;
    for (int k = 0; k < rows; ++k) s1 += redb[k * c4n];
    g.part_b[blk] = s1;
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

// Adjoint of pde_fields_kernel (src/pde.py:49-178 are differentiable in the reference): given
// upstream gradients of the three fields (any may be NULL = zero),
//   du = Lap*(g_lap + D g_res) + f'(u) g_res + sum_axis (G[k-1] - G[k+1]),  G = g_gm * (2 x the
// central difference) / 2 per axis,
// with Lap* the exact adjoint of the reflect-padded 5-point stencil (ghost row -1 = row 1 and
// row n = row n-2, so rows/columns 1 and n-2 take the boundary value twice) and the reflect
// central differences identically zero on the first/last row and column.
__global__ void pde_fields_bwd_kernel(const float* __restrict__ u0, const float* __restrict__ gl0,
                                      const float* __restrict__ gr0, const float* __restrict__ gg0, int B, int H,
                                      int W, float D, float a, float* __restrict__ du) {
  const int64_t HW = (int64_t)H * W, N = (int64_t)B * HW;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < N; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = e / HW;
    const int rem = (int)(e - b * HW), y = rem / W, x = rem - y * W;
    const float* u = u0 + b * HW;
    auto q = [&](int yy, int xx) -> float {  // Lap-adjoint input field, zero outside the image
      if (yy < 0 || yy >= H || xx < 0 || xx >= W) return 0.f;
      const int64_t o = b * HW + (int64_t)yy * W + xx;
      return (gl0 ? gl0[o] : 0.f) + (gr0 ? D * gr0[o] : 0.f);
    };
    float g = 0.f;
    if (gl0 || gr0) {
      const float qu = q(y - 1, x), qd = q(y + 1, x), ql = q(y, x - 1), qr = q(y, x + 1);
      g = (qu + qd) + (ql + qr) - 4.f * q(y, x);
      g += (y == 1 ? qu : 0.f) + (y == H - 2 ? qd : 0.f);
      g += (x == 1 ? ql : 0.f) + (x == W - 2 ? qr : 0.f);
    }
    if (gr0) {
      const float c = u[rem];
      g += gr0[e] * (c * (2.f * (1.f + a) - 3.f * c) - a);  // f'(u) = -3u^2 + 2(1+a)u - a
    }
    if (gg0) {
      const float* gg = gg0 + b * HW;
      auto gxw = [&](int yy, int xx) -> float {  // g_gm * gx at an interior column, else 0
        if (yy < 0 || yy >= H || xx < 1 || xx > W - 2) return 0.f;
        return gg[yy * W + xx] * (u[yy * W + xx + 1] - u[yy * W + xx - 1]);
      };
      auto gyw = [&](int yy, int xx) -> float {
        if (xx < 0 || xx >= W || yy < 1 || yy > H - 2) return 0.f;
        return gg[yy * W + xx] * (u[(yy + 1) * W + xx] - u[(yy - 1) * W + xx]);
      };
      // d(gx^2)/du[k] summed over the pixels whose difference touches k: 2 gx * (+-1/2) = +-gx
      g += 0.5f * ((gxw(y, x - 1) - gxw(y, x + 1)) + (gyw(y - 1, x) - gyw(y + 1, x)));
    }
    du[e] = g;
  }
}

static void loss_plan(int H, int W, int& tiles_x, int& tiles_y) {
  tiles_x = (W + LT_X - 1) / LT_X;
  tiles_y = (H + LT_Y - 1) / LT_Y;
}

}  // namespace pis

using namespace pis;

// workspace: [16 B reserved][fpart: nblk x 6 floats][ipart: nblk x 3 ints], nblk = the larger
// of the two plans
static int64_t loss_nblk(int B, int H, int W) {
  int tx, ty;
  loss_plan(H, W, tx, ty);
  int64_t n = (int64_t)B * tx * ty;
  if (loss_rows_ok(B, H, W)) n = std::max<int64_t>(n, (int64_t)B * cdiv(H, loss_rows(B, H, W)));
  return n;
}

extern "C" size_t pis_loss_ws(int B, int H, int W) {
  return 16 + (size_t)loss_nblk(B, H, W) * (6 * sizeof(float) + 3 * sizeof(int)) + 256;
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
  g.smooth = prm->smooth; g.D = prm->D; g.a = prm->a; g.eps = prm->eps;
  g.rx = (prm->flags & PIS_LOSS_NO_REACTION) ? 0.f : 1.f; g.thr = prm->thr;
  const int64_t nblk = loss_nblk(B, H, W);
  g.fpart = (float*)((char*)ws + 16);
  g.ipart = (int*)((char*)ws + 16 + (size_t)nblk * 6 * sizeof(float));
  const bool all = prm->flags & PIS_LOSS_ALL_TERMS;
  const bool rd = all || prm->rd_w > 0.f, pf = all || prm->pf_w > 0.f;
  hipStream_t s = (hipStream_t)stream;
  if (loss_rows_ok(B, H, W) && tune_get(PIS_TUNE_LOSS_ROWS) != 0) {
    LossRowArgs a{};
    a.g = g;
    a.rows = loss_rows(B, H, W);
    a.bands = (int)cdiv(H, a.rows);
    a.terms = out_terms; a.counts = counts; a.scores = scores;
    const dim3 grid(a.bands, B);
    const size_t smem = 0;
    if (rd && pf) hipLaunchKernelGGL((loss_fwd_rows_kernel<true, true>), grid, dim3(256), smem, s, a);
    else if (rd) hipLaunchKernelGGL((loss_fwd_rows_kernel<true, false>), grid, dim3(256), smem, s, a);
    else if (pf) hipLaunchKernelGGL((loss_fwd_rows_kernel<false, true>), grid, dim3(256), smem, s, a);
    else hipLaunchKernelGGL((loss_fwd_rows_kernel<false, false>), grid, dim3(256), smem, s, a);
    const int rc = launch_status("loss_fwd_rows");
    if (rc) return rc;
    hipLaunchKernelGGL(loss_finalize_rows_kernel, dim3(1), dim3(1024), 0, s, a);
    return launch_status("loss_finalize");
  }
  loss_plan(H, W, g.tiles_x, g.tiles_y);
  const dim3 grid(g.tiles_x, g.tiles_y, B);
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
  g.rx = (prm->flags & PIS_LOSS_NO_REACTION) ? 0.f : 1.f;
  g.terms = terms; g.grad_out = grad_out; g.dst = dst; g.chain = (flags & PIS_LOSS_CHAIN_SIGMOID) ? 1 : 0;
  int tx, ty;
  loss_plan(H, W, tx, ty);
  const dim3 grid(tx, ty, B);
  hipStream_t s = (hipStream_t)stream;
  const bool rd = prm->rd_w > 0.f, pf = prm->pf_w > 0.f;  // gradient only of terms in the total
  if (rd && pf) hipLaunchKernelGGL((loss_bwd_kernel<true, true>), grid, dim3(256), 0, s, g);
  else if (rd) hipLaunchKernelGGL((loss_bwd_kernel<true, false>), grid, dim3(256), 0, s, g);
  else if (pf) hipLaunchKernelGGL((loss_bwd_kernel<false, true>), grid, dim3(256), 0, s, g);
  else hipLaunchKernelGGL((loss_bwd_kernel<false, false>), grid, dim3(256), 0, s, g);
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

extern "C" int pis_pde_fields_bwd(const float* u, const float* g_lap, const float* g_residual,
                                  const float* g_gradmag2, int B, int H, int W, float D, float a, float* du,
                                  pis_stream_t stream) {
  PIS_CHECK_ARG(u && du && B > 0 && H >= 2 && W >= 2, "pis_pde_fields_bwd: bad arguments");
  const int64_t n = (int64_t)B * H * W;
  const int grid = (int)std::min<int64_t>(cdiv(n, 256), 8192);
  hipLaunchKernelGGL(pde_fields_bwd_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, u, g_lap, g_residual,
                     g_gradmag2, B, H, W, D, a, du);
  return launch_status("pde_fields_bwd");
}

static int head_loss_rows(int H, int W) { return std::max(1, std::min(H, 1024 / std::max(1, W))); }

static size_t head_loss_smem(int R, int W, bool rd) {
  const size_t f = (size_t)(R + 4) * (W + 4) + (rd ? (size_t)(R + 2) * (W + 2) : 0) + (size_t)R * W;
  return std::max(f * sizeof(float), (size_t)256 * 20);  // >= the reduction scratch
}

extern "C" size_t pis_head_loss_bwd_ws(int B, int H, int W, int C) {
  const int R = head_loss_rows(H, W);
  const size_t blocks = (size_t)B * ((H + R - 1) / R);
  return blocks * (C + 1) * sizeof(float) + 256;
}

extern "C" int pis_head_loss_bwd(const float* x, int ldx, const float* w, const float* u, const float* t,
                                 float* du_out, int B, int H, int W, int C,
                                 const pis_loss_params* prm, const float* terms, const float* grad_out,
                                 float* dx, int lddx, float* dw, float* db, int flags, void* ws,
                                 size_t ws_bytes, pis_stream_t stream) {
  PIS_CHECK_ARG(x && w && u && t && prm && terms && dx && dw && B > 0 && H >= 2 && W >= 2,
                "pis_head_loss_bwd: bad arguments");
  PIS_CHECK_ARG(C % 4 == 0 && C / 4 <= 256 && ldx % 4 == 0 && lddx % 4 == 0,
                "pis_head_loss_bwd: C and ld must be multiples of 4, C <= 1024");
  PIS_CHECK_ARG(W <= 1024, "pis_head_loss_bwd: W > 1024 (stage rows do not fit LDS); use pis_loss_bwd + pis_head_bwd");
  PIS_CHECK_ARG(ws && ws_bytes >= pis_head_loss_bwd_ws(B, H, W, C), "pis_head_loss_bwd: workspace too small");
  HeadLossArgs g{};
  g.x = x; g.ldx = ldx; g.w = w; g.u = u; g.t = t; g.du_out = du_out;
  g.B = B; g.H = H; g.W = W; g.C = C; g.R = head_loss_rows(H, W);
  g.dice_w = prm->dice_w; g.bce_w = prm->bce_w; g.rd_w = prm->rd_w; g.pf_w = prm->pf_w;
  g.smooth = prm->smooth; g.D = prm->D; g.a = prm->a; g.eps = prm->eps;
  g.rx = (prm->flags & PIS_LOSS_NO_REACTION) ? 0.f : 1.f;
  g.terms = terms; g.grad_out = grad_out; g.dx = dx; g.lddx = lddx;
  const dim3 grid((H + g.R - 1) / g.R, B);
  g.part = (float*)ws;
  g.part_b = g.part + (size_t)grid.x * grid.y * C;
  hipStream_t s = (hipStream_t)stream;
  const bool rd = prm->rd_w > 0.f, pf = prm->pf_w > 0.f;
  const size_t smem = head_loss_smem(g.R, W, rd);
  if (rd && pf) hipLaunchKernelGGL((head_loss_bwd_kernel<true, true>), grid, dim3(256), smem, s, g);
  else if (rd) hipLaunchKernelGGL((head_loss_bwd_kernel<true, false>), grid, dim3(256), smem, s, g);
  else if (pf) hipLaunchKernelGGL((head_loss_bwd_kernel<false, true>), grid, dim3(256), smem, s, g);
  else hipLaunchKernelGGL((head_loss_bwd_kernel<false, false>), grid, dim3(256), smem, s, g);
  int rc = launch_status("head_loss_bwd");
  const int acc = flags & PIS_ACCUMULATE;
  if (!rc) rc = reduce_slabs(g.part, (int)(grid.x * grid.y), C, dw, acc, s);
  if (!rc && db) rc = reduce_slabs(g.part_b, (int)(grid.x * grid.y), 1, db, acc, s);
  return rc;
}
