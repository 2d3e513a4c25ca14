// Bandwidth-bound kernels of the step: 2x2 max pooling (src/unet.py:126),
// the 1x1 output head + sigmoid (src/unet.py:157,206-210) and decoupled AdamW
// (src/train.py:658-662). NHWC fp32, 16-byte vector accesses.
#include "common.h"

namespace pis {

__global__ void maxpool_fwd_kernel(const float* __restrict__ x, int ldx, float* __restrict__ y,
                                   int B, int Ho, int Wo, int C) {
  const int c4n = C / 4;
  const int64_t n = (int64_t)B * Ho * Wo * c4n;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int c4 = (int)(e % c4n);
    const int64_t q = e / c4n;  // pooled pixel
    const int wo = (int)(q % Wo);
    const int64_t bh = q / Wo;
    const int ho = (int)(bh % Ho);
    const int b = (int)(bh / Ho);
    const int W = 2 * Wo;
    const int64_t p00 = ((int64_t)b * 2 * Ho + 2 * ho) * W + 2 * wo;
    const f32x4 v0 = *reinterpret_cast<const f32x4*>(x + p00 * ldx + 4 * c4);
    const f32x4 v1 = *reinterpret_cast<const f32x4*>(x + (p00 + 1) * ldx + 4 * c4);
    const f32x4 v2 = *reinterpret_cast<const f32x4*>(x + (p00 + W) * ldx + 4 * c4);
    const f32x4 v3 = *reinterpret_cast<const f32x4*>(x + (p00 + W + 1) * ldx + 4 * c4);
    f32x4 m;
#pragma unroll
    for (int j = 0; j < 4; ++j) m[j] = fmaxf(fmaxf(v0[j], v1[j]), fmaxf(v2[j], v3[j]));
    *reinterpret_cast<f32x4*>(y + q * C + 4 * c4) = m;
  }
}

// dx = (dskip + route(dy)) * (x > 0); route = first max in (0,0),(0,1),(1,0),(1,1)
// order, the tie-break of ATen's max_pool2d_with_indices.
// I: index type of the element loop (int when the item count fits: 32-bit divisions are a few
// instructions, 64-bit ones a software routine per item)
template <typename I>
__global__ void maxpool_bwd_kernel(const float* __restrict__ x, int ldx, const float* __restrict__ dy,
                                   const float* __restrict__ dskip, int ldskip,
                                   float* __restrict__ dx, int lddx, int B, int Ho, int Wo, int C) {
  const int c4n = C / 4;
  const I n = (I)B * Ho * Wo * c4n;
  for (I e = (I)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (I)gridDim.x * blockDim.x) {
    const int c4 = (int)(e % c4n);
    const I q = e / c4n;
    const int wo = (int)(q % Wo);
    const I bh = q / Wo;
    const int ho = (int)(bh % Ho);
    const int b = (int)(bh / Ho);
    const int W = 2 * Wo;
    const int64_t p00 = ((int64_t)b * 2 * Ho + 2 * ho) * W + 2 * wo;
    const int64_t pix[4] = {p00, p00 + 1, p00 + W, p00 + W + 1};
    f32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = *reinterpret_cast<const f32x4*>(x + pix[k] * ldx + 4 * c4);
    const f32x4 g = *reinterpret_cast<const f32x4*>(dy + q * C + 4 * c4);
    int arg[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int a = 0;
      float best = v[0][j];
#pragma unroll
      for (int k = 1; k < 4; ++k)
        if (v[k][j] > best) { best = v[k][j]; a = k; }
      arg[j] = a;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f32x4 o = dskip ? *reinterpret_cast<const f32x4*>(dskip + pix[k] * ldskip + 4 * c4)
                      : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (arg[j] == k) o[j] += g[j];
        o[j] = v[k][j] > 0.f ? o[j] : 0.f;
      }
      *reinterpret_cast<f32x4*>(dx + pix[k] * lddx + 4 * c4) = o;
    }
  }
}

// head fwd: 16 lanes per pixel (4 pixels per wave-instruction), float4 each
__global__ __launch_bounds__(256) void head_fwd_kernel(const float* __restrict__ x, int ldx,
                                                       const float* __restrict__ w,
                                                       const float* __restrict__ b,
                                                       float* __restrict__ z, float* __restrict__ u,
                                                       int64_t npix, int C) {
  const int sub = threadIdx.x & 15;
  const int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const bool ok = p < npix;
  float s = 0.f;
  if (ok)
    for (int c = 4 * sub; c < C; c += 64) {
      const f32x4 xv = *reinterpret_cast<const f32x4*>(x + p * ldx + c);
      const f32x4 wv = *reinterpret_cast<const f32x4*>(w + c);
      s = fmaf(xv[0], wv[0], s);
      s = fmaf(xv[1], wv[1], s);
      s = fmaf(xv[2], wv[2], s);
      s = fmaf(xv[3], wv[3], s);
    }
  s = group16_sum(s);
  if (ok && sub == 0) {
    const float zz = s + b[0];
    if (z) z[p] = zz;
    u[p] = 1.f / (1.f + expf(-zz));
  }
}

// head fwd for C == 64 (the U-Net's head): the same 16-lane pixel groups, each taking PP pixels
// G groups apart (G = the grid's group count) with all PP float4 loads issued before the sums —
// PP x the bytes in flight of head_fwd_kernel's one load per thread; per pixel the same
// fixed-order sum (group16_sum), so z and u are bitwise those of head_loss_fwd_kernel
template <int PP>
__global__ __launch_bounds__(256) void head_fwd64_kernel(const float* __restrict__ x, int ldx,
                                                         const float* __restrict__ w,
                                                         const float* __restrict__ b,
                                                         float* __restrict__ z, float* __restrict__ u,
                                                         int64_t npix) {
  const int sub = threadIdx.x & 15;
  const int64_t q = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const int64_t G = ((int64_t)gridDim.x * blockDim.x) >> 4;
  const f32x4 wv = *reinterpret_cast<const f32x4*>(w + 4 * sub);
  f32x4 xv[PP];
#pragma unroll
  for (int k = 0; k < PP; ++k) {
    const int64_t p = q + k * G;
    xv[k] = p < npix ? *reinterpret_cast<const f32x4*>(x + p * ldx + 4 * sub) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int k = 0; k < PP; ++k) {
    const int64_t p = q + k * G;
    float s = 0.f;
    s = fmaf(xv[k][0], wv[0], s);
    s = fmaf(xv[k][1], wv[1], s);
    s = fmaf(xv[k][2], wv[2], s);
    s = fmaf(xv[k][3], wv[3], s);
    s = group16_sum(s);  // the same fixed order as head_loss_fwd_kernel (csrc/loss.hip): bitwise equal z
    if (p < npix && sub == 0) {
      const float zz = s + b[0];
      if (z) z[p] = zz;
      u[p] = 1.f / (1.f + expf(-zz));
    }
  }
}

// head bwd: d = g u (1-u) (or g); dx[p][c] = d w[c] (x[p][c] > 0); per-block partial dw[c], db
__global__ __launch_bounds__(256) void head_bwd_kernel(const float* __restrict__ x, int ldx,
                                                       const float* __restrict__ w,
                                                       const float* __restrict__ gin,
                                                       const float* __restrict__ u,
                                                       float* __restrict__ dx, int lddx,
                                                       int64_t npix, int C, int64_t pix_per_block,
                                                       float* __restrict__ part,
                                                       float* __restrict__ part_b) {
  // C % 4 == 0, C <= 1024: lane group of C/4 threads covers one pixel
  const int c4n = C / 4;
  const int rows = 256 / c4n;
  const int r = threadIdx.x / c4n, c4 = threadIdx.x - r * c4n;
  const int64_t p0 = (int64_t)blockIdx.x * pix_per_block;
  const int64_t p1 = min(npix, p0 + pix_per_block);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float accb = 0.f;
  if (r < rows) {
    const f32x4 wv = *reinterpret_cast<const f32x4*>(w + 4 * c4);
    for (int64_t p = p0 + r; p < p1; p += rows) {
      float d = gin[p];
      if (u) { const float uu = u[p]; d = d * (1.f - uu) * uu; }
      if (c4 == 0) accb += d;
      const f32x4 xv = *reinterpret_cast<const f32x4*>(x + p * ldx + 4 * c4);
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = xv[j] > 0.f ? d * wv[j] : 0.f;
        acc[j] = fmaf(d, xv[j], acc[j]);
      }
      *reinterpret_cast<f32x4*>(dx + p * lddx + 4 * c4) = o;
    }
  }
  __shared__ f32x4 red[256];
  __shared__ float redb[256];
  red[threadIdx.x] = acc;
  redb[threadIdx.x] = accb;
  __syncthreads();
  if ((int)threadIdx.x < c4n) {
    f32x4 t = red[threadIdx.x];
    for (int k = 1; k < rows; ++k) t += red[k * c4n + threadIdx.x];
    *reinterpret_cast<f32x4*>(part + (size_t)blockIdx.x * C + 4 * threadIdx.x) = t;
  }
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < rows; ++k) t += redb[k * c4n];
    part_b[blockIdx.x] = t;
  }
}

__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                             float* __restrict__ m, float* __restrict__ v, int64_t n, float decay,
                             float omb1, float beta2, float omb2, float eps, float step_size,
                             float bc2_sqrt, float grad_scale) {
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4 + (n - n4 * 4);
       i += (int64_t)gridDim.x * blockDim.x) {
    if (i < n4) {
      f32x4 pp = reinterpret_cast<f32x4*>(p)[i];
      f32x4 gg = reinterpret_cast<const f32x4*>(g)[i];
      f32x4 mm = reinterpret_cast<f32x4*>(m)[i];
      f32x4 vv = reinterpret_cast<f32x4*>(v)[i];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float gj = gg[j] * grad_scale;
        pp[j] = pp[j] * decay;
        mm[j] = mm[j] + omb1 * (gj - mm[j]);
        vv[j] = vv[j] * beta2 + omb2 * gj * gj;
        const float denom = sqrtf(vv[j]) / bc2_sqrt + eps;
        pp[j] = pp[j] + (-step_size) * (mm[j] / denom);
      }
      reinterpret_cast<f32x4*>(p)[i] = pp;
      reinterpret_cast<f32x4*>(m)[i] = mm;
      reinterpret_cast<f32x4*>(v)[i] = vv;
    } else {
      const int64_t k = n4 * 4 + (i - n4);
      const float gj = g[k] * grad_scale;
      float pp = p[k] * decay;
      const float mm = m[k] + omb1 * (gj - m[k]);
      const float vv = v[k] * beta2 + omb2 * gj * gj;
      pp = pp + (-step_size) * (mm / (sqrtf(vv) / bc2_sqrt + eps));
      p[k] = pp; m[k] = mm; v[k] = vv;
    }
  }
}

int reduce_slabs(const float* part, int splits, int64_t n, float* dst, int accumulate, hipStream_t s);
int reduce_slabs2(const float* part, int splits, int64_t n, float* dst, const float* part_b, int splits_b,
                  int64_t n_b, float* dst_b, int accumulate, hipStream_t s);
int colsum(const float* src, int ld, int64_t npix, int C, float* out, int accumulate, void* ws,
           size_t ws_bytes, hipStream_t s);
size_t colsum_ws(int64_t npix, int C);

static int64_t head_pix_per_block(int64_t npix) { return std::max<int64_t>(256, cdiv(npix, 2048)); }

// Bandwidth probes for the loss roofline (bench.py 'roofline_loss'): the least a kernel can take to
// move the loss's algorithmic bytes at its size, under the same cold-cache protocol — one launch,
// float4 grid-stride, a read of a and b reduced to one partial per block (the forward's 8 B/px) or
// dst = a + b (the backward's 12 B/px).
__global__ __launch_bounds__(256) void stream_probe_kernel(const f32x4* __restrict__ a, const f32x4* __restrict__ b,
                                                           f32x4* __restrict__ dst, int64_t n4, float* partial) {
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const f32x4 v = a[i] + b[i];
    if (dst) dst[i] = v;
    else acc += v[0] + v[1] + v[2] + v[3];
  }
  if (!dst) {
    __shared__ float red[4];
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) partial[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
  }
}

// Access-order probe (tooling): a 1024-thread block per CU reads 16-KB chunks (one float4 per lane),
// eight chunks in flight per lane. mode 0 sweeps: pass i of block p reads chunk i * grid + p, so the
// grid's concurrent reads sit in one window; mode 1 bands: block p reads its own contiguous run of
// chunks (the row-band kernels' order: concurrent reads spread over the whole buffer).
__global__ __launch_bounds__(1024) void band_probe_kernel(const f32x4* __restrict__ a, int64_t nchunk, int mode,
                                                          float* partial) {
  const int64_t per = nchunk / gridDim.x;
  float acc = 0.f;
  for (int64_t i = 0; i + 8 <= per; i += 8) {
    f32x4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t c = mode == 0 ? (i + u) * gridDim.x + blockIdx.x : blockIdx.x * per + i + u;
      v[u] = a[c * 1024 + threadIdx.x];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += (v[u][0] + v[u][1]) + (v[u][2] + v[u][3]);
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) partial[blockIdx.x * 16 + (threadIdx.x >> 6)] = acc;
}

}  // namespace pis

using namespace pis;

static int grid_for(int64_t work) { return (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(work, 256), 8192)); }

extern "C" int pis_maxpool2x2_fwd(const float* x, int ldx, float* y, int B, int H, int W, int C,
                                  pis_stream_t stream) {
  PIS_CHECK_ARG(x && y && B > 0 && H >= 2 && W >= 2 && C > 0, "pis_maxpool2x2_fwd: bad arguments");
  PIS_CHECK_ARG(H % 2 == 0 && W % 2 == 0 && C % 4 == 0 && ldx % 4 == 0,
                "pis_maxpool2x2_fwd: H, W even and C, ldx multiples of 4 required");
  const int64_t work = (int64_t)B * (H / 2) * (W / 2) * (C / 4);
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)stream,
                     x, ldx, y, B, H / 2, W / 2, C);
  return launch_status("maxpool2x2_fwd");
}

extern "C" int pis_maxpool2x2_bwd(const float* x, int ldx, const float* dy, const float* dskip,
                                  int ldskip, float* dx, int lddx, int B, int H, int W, int C,
                                  pis_stream_t stream) {
  PIS_CHECK_ARG(x && dy && dx && B > 0 && H >= 2 && W >= 2 && C > 0, "pis_maxpool2x2_bwd: bad arguments");
  PIS_CHECK_ARG(H % 2 == 0 && W % 2 == 0 && C % 4 == 0 && ldx % 4 == 0 && lddx % 4 == 0 &&
                    (!dskip || ldskip % 4 == 0),
                "pis_maxpool2x2_bwd: H, W even and C, ld multiples of 4 required");
  const int64_t work = (int64_t)B * (H / 2) * (W / 2) * (C / 4);
  if (work < (int64_t)1 << 30)
    hipLaunchKernelGGL(maxpool_bwd_kernel<int>, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)stream,
                       x, ldx, dy, dskip, ldskip, dx, lddx, B, H / 2, W / 2, C);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<int64_t>, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)stream,
                       x, ldx, dy, dskip, ldskip, dx, lddx, B, H / 2, W / 2, C);
  return launch_status("maxpool2x2_bwd");
}

extern "C" int pis_head_fwd(const float* x, int ldx, const float* w, const float* b, float* z,
                            float* u, int64_t npix, int C, pis_stream_t stream) {
  PIS_CHECK_ARG(x && w && b && u && npix > 0 && C > 0 && C % 4 == 0 && ldx % 4 == 0,
                "pis_head_fwd: bad arguments");
  if (C == 64) {  // 4 pixels per 16-lane group
    hipLaunchKernelGGL(head_fwd64_kernel<4>, dim3((unsigned)cdiv(cdiv(npix, 4) * 16, 256)), dim3(256), 0,
                       (hipStream_t)stream, x, ldx, w, b, z, u, npix);
    return launch_status("head_fwd");
  }
  hipLaunchKernelGGL(head_fwd_kernel, dim3((unsigned)cdiv(npix * 16, 256)), dim3(256), 0,
                     (hipStream_t)stream, x, ldx, w, b, z, u, npix, C);
  return launch_status("head_fwd");
}

extern "C" size_t pis_head_bwd_ws(int64_t npix, int C) {
  const int64_t blocks = cdiv(npix, head_pix_per_block(npix));
  return (size_t)blocks * (C + 1) * sizeof(float) + 256;
}

extern "C" int pis_head_bwd(const float* x, int ldx, const float* w, const float* g, const float* u,
                            float* dx, int lddx, float* dw, float* db, int64_t npix, int C,
                            int flags, void* ws, size_t ws_bytes, pis_stream_t stream) {
  PIS_CHECK_ARG(x && w && g && dx && dw && npix > 0 && C % 4 == 0 && C / 4 <= 256 &&
                    ldx % 4 == 0 && lddx % 4 == 0,
                "pis_head_bwd: bad arguments");
  PIS_CHECK_ARG(ws_bytes >= pis_head_bwd_ws(npix, C), "pis_head_bwd: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int acc = flags & PIS_ACCUMULATE;
  const int64_t ppb = head_pix_per_block(npix);
  const int blocks = (int)cdiv(npix, ppb);
  float* part = (float*)ws;
  float* part_b = part + (size_t)blocks * C;
  hipLaunchKernelGGL(head_bwd_kernel, dim3(blocks), dim3(256), 0, s, x, ldx, w, g, u, dx, lddx, npix,
                     C, ppb, part, part_b);
  int rc = launch_status("head_bwd");
  if (!rc) rc = reduce_slabs2(part, blocks, C, dw, db ? part_b : nullptr, blocks, 1, db, acc, s);
  return rc;
}

extern "C" int pis_adamw_step(float* p, const float* g, float* m, float* v, int64_t n, double lr,
                              double beta1, double beta2, double eps, double weight_decay,
                              double step_size, double bc2_sqrt, double grad_scale,
                              pis_stream_t stream) {
  // scalars are rounded to fp32 exactly as torch's single-tensor AdamW rounds its Python floats
  PIS_CHECK_ARG(p && g && m && v && n >= 0, "pis_adamw_step: bad arguments");
  PIS_CHECK_ARG(((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) % 16 == 0,
                "pis_adamw_step: buffers must be 16-byte aligned");
  if (n == 0) return PIS_OK;
  const float decay = (float)(1.0 - lr * weight_decay);
  const float omb1 = (float)(1.0 - beta1);
  const float omb2 = (float)(1.0 - beta2);
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(n / 4 + 4)), dim3(256), 0, (hipStream_t)stream, p,
                     g, m, v, n, decay, omb1, (float)beta2, omb2, (float)eps, (float)step_size,
                     (float)bc2_sqrt, (float)grad_scale);
  return launch_status("adamw");
}

extern "C" int pis_debug_stream_probe(const float* a, const float* b, float* dst, int64_t n, float* partial,
                                      int grid, pis_stream_t stream) {
  PIS_CHECK_ARG(a && b && n > 0 && n % 4 == 0 && grid > 0 && (dst || partial), "pis_debug_stream_probe: bad arguments");
  hipLaunchKernelGGL(stream_probe_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const f32x4*>(a), reinterpret_cast<const f32x4*>(b),
                     reinterpret_cast<f32x4*>(dst), n / 4, partial);
  return launch_status("stream_probe");
}

extern "C" int pis_debug_band_probe(const float* a, int64_t n, int mode, float* partial, int grid,
                                    pis_stream_t stream) {
  PIS_CHECK_ARG(a && partial && grid > 0 && n % 4096 == 0 && (mode == 0 || mode == 1),
                "pis_debug_band_probe: bad arguments");
  hipLaunchKernelGGL(band_probe_kernel, dim3(grid), dim3(1024), 0, (hipStream_t)stream,
                     reinterpret_cast<const f32x4*>(a), n / 4096, mode, partial);
  return launch_status("band_probe");
}
