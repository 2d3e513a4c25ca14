// Weight-gradient GEMMs (fp32 MFMA) for src/unet.py's 3x3 convs and 2x2
// transposed convs, plus channel sums for bias gradients.
//
//   C[m'][n'] = sum_p A(p, m') * B(p, n')       p = pixel of the reduction grid
//
// The pixel reduction (up to B*H*W = 2.1M at 512^2) is split over blocks
// ("splits"); every block writes its partial C tile to a slab and a second
// kernel sums the slabs in a fixed order, so the result is deterministic and
// each fp32 accumulation chain is at most `pix_per_split` long.
//
// conv3x3:  m' = n (Cout),        A(p, n)     = dz[p][n]
//           n' = (tap, c),        B(p, tap,c) = x[p + off(tap)][c]    (zero pad)
// convT2x2: m' = (i, j, o),       A(p, ijo)   = dy[(2h+i, 2w+j)][o]
//           n' = c,               B(p, c)     = x[p][c]
#include "common.h"

namespace pis {

struct WgradArgs {
  const float* a; int lda; int a_up2; int Ca;   // Ca: channels per (i,j) group when a_up2
  const float* b; int ldb; int b_conv3; int Cb;  // Cb: channels per tap when b_conv3
  int B, H, W;                                   // reduction pixel grid
  int P;                                         // B*H*W
  int Mp, Np;                                    // output dims
  int pix_per_split;
  float* part;                                   // [splits][Mp][Np]
};

template <int BM, int BN>
__global__ __launch_bounds__(256) void wgrad_f32_kernel(WgradArgs g) {
  constexpr int BKP = 16;                     // pixels per stage
  constexpr int TM = BM / 64, TN = BN / 64;   // 32x32 tiles per wave
  constexpr int AL = BKP * BM / 4 / 256, BL = BKP * BN / 4 / 256;
  __shared__ __attribute__((aligned(16))) float sA[2][BKP * BM];
  __shared__ __attribute__((aligned(16))) float sB[2][BKP * BN];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntm = g.Mp / BM, ntn = g.Np / BN;
  const int tiles = ntm * ntn;
  const int split = blockIdx.x / tiles;
  const int tile = blockIdx.x - split * tiles;
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const int p_begin = split * g.pix_per_split;
  const int p_end = min(g.P, p_begin + g.pix_per_split);

  // tap of this tile (tiles never straddle a tap)
  int a_dr = 0, a_ds = 0, a_c0 = m0;
  if (g.a_up2) { const int ij = m0 / g.Ca; a_dr = ij >> 1; a_ds = ij & 1; a_c0 = m0 - ij * g.Ca; }
  int b_dr = 0, b_ds = 0, b_c0 = n0;
  if (g.b_conv3) { const int t = n0 / g.Cb; b_dr = t / 3 - 1; b_ds = t % 3 - 1; b_c0 = n0 - t * g.Cb; }
  const int HW = g.H * g.W;

  f32x4 ra[AL], rb[BL];
  auto gload = [&](int p0) {
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int idx = tid + i * 256;
      const int prow = idx / (BM / 4), c = (idx % (BM / 4)) * 4;
      const int p = p0 + prow;
      ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (p < p_end) {
        size_t pix = p;
        if (g.a_up2) {
          const int bb = p / HW, rem = p - bb * HW, h = rem / g.W, w = rem - h * g.W;
          pix = ((size_t)bb * 2 * g.H + 2 * h + a_dr) * (2 * g.W) + 2 * w + a_ds;
        }
        ra[i] = *reinterpret_cast<const f32x4*>(g.a + pix * g.lda + a_c0 + c);
      }
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int idx = tid + i * 256;
      const int prow = idx / (BN / 4), c = (idx % (BN / 4)) * 4;
      const int p = p0 + prow;
      rb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (p < p_end) {
        bool ok = true;
        size_t pix = p;
        if (g.b_conv3) {
          const int bb = p / HW, rem = p - bb * HW, h = rem / g.W, w = rem - h * g.W;
          const int hs = h + b_dr, ws = w + b_ds;
          ok = hs >= 0 && hs < g.H && ws >= 0 && ws < g.W;
          pix = ((size_t)bb * g.H + hs) * g.W + ws;
        }
        if (ok) rb[i] = *reinterpret_cast<const f32x4*>(g.b + pix * g.ldb + b_c0 + c);
      }
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AL; ++i) *reinterpret_cast<f32x4*>(&sA[buf][(tid + i * 256) * 4]) = ra[i];
#pragma unroll
    for (int i = 0; i < BL; ++i) *reinterpret_cast<f32x4*>(&sB[buf][(tid + i * 256) * 4]) = rb[i];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int li = lane & 31, lh = lane >> 5;
  const int nst = (p_end - p_begin + BKP - 1) / BKP;
  if (nst > 0) {
    gload(p_begin);
    lstore(0);
  }
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    if (st + 1 < nst) gload(p_begin + (st + 1) * BKP);
    const float* As = sA[cur];
    const float* Bs = sB[cur];
#pragma unroll
    for (int kk = 0; kk < BKP / 2; ++kk) {
      const int prow = 2 * kk + lh;
      float af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a] = As[prow * BM + wm * (BM / 2) + a * 32 + li];
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[b] = Bs[prow * BN + wn * (BN / 2) + b * 32 + li];
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a], bf[b], acc[a][b], 0, 0, 0);
    }
    if (st + 1 < nst) lstore(cur ^ 1);
    __syncthreads();
  }

  float* out = g.part + (size_t)split * g.Mp * g.Np;
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int n = n0 + wn * (BN / 2) + b * 32 + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * (BM / 2) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        out[(size_t)m * g.Np + n] = acc[a][b][r];
      }
    }
}

// dst[i] = (acc ? dst[i] : 0) + sum_s part[s][i], fixed order (deterministic)
__global__ void reduce_slabs_kernel(const float* __restrict__ part, int splits, int64_t n,
                                    float* __restrict__ dst, int accumulate) {
  const int64_t n4 = n / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    f32x4 s = accumulate ? reinterpret_cast<f32x4*>(dst)[i] : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < splits; ++k) s += reinterpret_cast<const f32x4*>(part + (size_t)k * n)[i];
    reinterpret_cast<f32x4*>(dst)[i] = s;
  }
  const int64_t tail0 = n4 * 4;
  for (int64_t i = tail0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float s = accumulate ? dst[i] : 0.f;
    for (int k = 0; k < splits; ++k) s += part[(size_t)k * n + i];
    dst[i] = s;
  }
}

int reduce_slabs(const float* part, int splits, int64_t n, float* dst, int accumulate,
                 hipStream_t s) {
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(n / 4 + 1, 256), 2048));
  hipLaunchKernelGGL(reduce_slabs_kernel, dim3(grid), dim3(256), 0, s, part, splits, n, dst,
                     accumulate);
  return launch_status("reduce_slabs");
}

// Column sums: part[split][c] = sum_{p in split} src[p*ld + c]
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ src, int ld,
                                                     int64_t npix, int C, int64_t pix_per_split,
                                                     float* __restrict__ part) {
  // C % 4 == 0 and C/4 <= 256 : lanes cover the channels, rows cover pixels
  const int c4n = C / 4;
  const int rows = 256 / c4n;
  const int tid = threadIdx.x;
  const int r = tid / c4n, c4 = tid - r * c4n;
  const int64_t p0 = (int64_t)blockIdx.x * pix_per_split;
  const int64_t p1 = min(npix, p0 + pix_per_split);
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (r < rows)
    for (int64_t p = p0 + r; p < p1; p += rows) s += *reinterpret_cast<const f32x4*>(src + p * ld + 4 * c4);
  __shared__ f32x4 red[256];
  red[tid] = s;
  __syncthreads();
  if (tid < c4n) {
    f32x4 t = red[tid];
    for (int k = 1; k < rows; ++k) t += red[k * c4n + tid];
    *reinterpret_cast<f32x4*>(part + (size_t)blockIdx.x * C + 4 * tid) = t;
  }
}

// Scalar column sum for C not a multiple of 4 (C = 1 head bias): one sum per block
__global__ __launch_bounds__(256) void colsum1_kernel(const float* __restrict__ src, int ld,
                                                      int64_t npix, int C, int64_t pix_per_split,
                                                      float* __restrict__ part) {
  const int64_t p0 = (int64_t)blockIdx.x * pix_per_split;
  const int64_t p1 = min(npix, p0 + pix_per_split);
  __shared__ float red[4];
  for (int c = 0; c < C; ++c) {
    float s = 0.f;
    for (int64_t p = p0 + threadIdx.x; p < p1; p += 256) s += src[p * ld + c];
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) part[(size_t)blockIdx.x * C + c] = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
  }
}

static void colsum_plan(int64_t npix, int C, int& splits, int64_t& pps) {
  pps = std::max<int64_t>(1024, cdiv(npix, 1024));
  splits = (int)cdiv(npix, pps);
}

int colsum(const float* src, int ld, int64_t npix, int C, float* out, int accumulate, void* ws,
           size_t ws_bytes, hipStream_t s) {
  int splits;
  int64_t pps;
  colsum_plan(npix, C, splits, pps);
  if (ws_bytes < (size_t)splits * C * sizeof(float)) {
    set_error("colsum: workspace too small");
    return PIS_ERR_WORKSPACE;
  }
  float* part = (float*)ws;
  if (C % 4 == 0 && C / 4 <= 256) {
    hipLaunchKernelGGL(colsum_kernel, dim3(splits), dim3(256), 0, s, src, ld, npix, C, pps, part);
  } else {
    hipLaunchKernelGGL(colsum1_kernel, dim3(splits), dim3(256), 0, s, src, ld, npix, C, pps, part);
  }
  int rc = launch_status("colsum");
  if (rc) return rc;
  return reduce_slabs(part, splits, C, out, accumulate, s);
}

size_t colsum_ws(int64_t npix, int C) {
  int splits;
  int64_t pps;
  colsum_plan(npix, C, splits, pps);
  return (size_t)splits * C * sizeof(float);
}

// ---- wgrad planning -------------------------------------------------------
struct WgradPlan {
  int bm, bn, splits, pps;
  size_t part_bytes;
};

static WgradPlan plan_wgrad(int Mp, int Np, int P, int group_m, int group_n) {
  // tile sizes must divide the per-tap group so tiles never straddle a tap
  WgradPlan p{};
  p.bm = (Mp % 128 == 0 && group_m % 128 == 0) ? 128 : 64;
  p.bn = (Np % 128 == 0 && group_n % 128 == 0) ? 128 : 64;
  const int tiles = (Mp / p.bm) * (Np / p.bn);
  // >= ~2 blocks per CU, fp32 chains of at most 8192 pixels, at least 64 pixels per split
  const int64_t want_splits = std::max<int64_t>(1, cdiv(512, tiles));
  int64_t pps = std::max<int64_t>(64, cdiv(P, want_splits));
  pps = std::min<int64_t>(pps, 8192);
  pps = cdiv(pps, 16) * 16;
  p.pps = (int)pps;
  p.splits = (int)cdiv(P, pps);
  p.part_bytes = (size_t)p.splits * Mp * Np * sizeof(float);
  return p;
}

static int run_wgrad(const WgradArgs& base, const WgradPlan& pl, float* dst, int accumulate,
                     hipStream_t s) {
  WgradArgs a = base;
  a.pix_per_split = pl.pps;
  const int tiles = (a.Mp / pl.bm) * (a.Np / pl.bn);
  const dim3 grid(tiles * pl.splits);
  if (pl.bm == 128 && pl.bn == 128)
    hipLaunchKernelGGL((wgrad_f32_kernel<128, 128>), grid, dim3(256), 0, s, a);
  else if (pl.bm == 128)
    hipLaunchKernelGGL((wgrad_f32_kernel<128, 64>), grid, dim3(256), 0, s, a);
  else if (pl.bn == 128)
    hipLaunchKernelGGL((wgrad_f32_kernel<64, 128>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((wgrad_f32_kernel<64, 64>), grid, dim3(256), 0, s, a);
  int rc = launch_status("wgrad_f32");
  if (rc) return rc;
  return reduce_slabs(a.part, pl.splits, (int64_t)a.Mp * a.Np, dst, accumulate, s);
}

// Cin == 1 conv wgrad (enc1.conv0): dw[n][t] = sum_p dz[p][n] * x[p+off(t)]
__global__ __launch_bounds__(256) void wgrad_c1_kernel(const float* __restrict__ x, int ldx,
                                                       const float* __restrict__ dz, int ldz,
                                                       int B, int H, int W, int Cout,
                                                       int pix_per_split, float* __restrict__ part) {
  // thread owns output channel n = tid % Cout for a subset of rows; Cout <= 256
  const int HW = H * W, P = B * HW;
  const int p0 = blockIdx.x * pix_per_split, p1 = min(P, p0 + pix_per_split);
  const int rows = 256 / Cout;
  const int n = threadIdx.x % Cout, r = threadIdx.x / Cout;
  float s[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) s[t] = 0.f;
  if (r < rows) {
    for (int p = p0 + r; p < p1; p += rows) {
      const int bb = p / HW, rem = p - bb * HW, h = rem / W, w = rem - h * W;
      const float d = dz[(size_t)p * ldz + n];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int hh = h + t / 3 - 1, ww = w + t % 3 - 1;
        const float xv = (hh >= 0 && hh < H && ww >= 0 && ww < W) ? x[((size_t)bb * HW + hh * W + ww) * ldx] : 0.f;
        s[t] = fmaf(d, xv, s[t]);
      }
    }
  }
  __shared__ float red[256 * 9];
#pragma unroll
  for (int t = 0; t < 9; ++t) red[t * 256 + threadIdx.x] = s[t];
  __syncthreads();
  for (int o = threadIdx.x; o < Cout * 9; o += 256) {
    const int nn = o / 9, t = o - nn * 9;
    float v = 0.f;
    for (int k = 0; k < rows; ++k) v += red[t * 256 + k * Cout + nn];
    part[(size_t)blockIdx.x * Cout * 9 + o] = v;
  }
}

}  // namespace pis

using namespace pis;

extern "C" size_t pis_colsum_ws(int64_t npix, int C) { return colsum_ws(npix, C); }

extern "C" int pis_colsum(const float* src, int ld, int64_t npix, int C, float* out, int flags,
                          void* ws, size_t ws_bytes, pis_stream_t stream) {
  PIS_CHECK_ARG(src && out && npix > 0 && C > 0, "pis_colsum: bad arguments");
  PIS_CHECK_ARG(C % 4 != 0 || ld % 4 == 0, "pis_colsum: ld must be a multiple of 4");
  return colsum(src, ld, npix, C, out, flags & PIS_ACCUMULATE, ws, ws_bytes, (hipStream_t)stream);
}

static size_t c1_part_bytes(int P, int Cout, int& splits, int& pps) {
  pps = std::max(1024, (int)cdiv(P, 512));
  splits = (int)cdiv(P, pps);
  return (size_t)splits * Cout * 9 * sizeof(float);
}

extern "C" size_t pis_conv3x3_wgrad_ws(int B, int H, int W, int Cin, int Cout) {
  const int P = B * H * W;
  size_t wbytes;
  if (Cin == 1) {
    int sp, pps;
    wbytes = c1_part_bytes(P, Cout, sp, pps);
  } else {
    wbytes = plan_wgrad(Cout, 9 * Cin, P, Cout, Cin).part_bytes;
  }
  return std::max(wbytes, colsum_ws(P, Cout)) + 256;
}

extern "C" int pis_conv3x3_wgrad(const float* x, int ldx, const float* dz, int ldz, float* dw_krsc,
                                 float* db, int B, int H, int W, int Cin, int Cout, int flags,
                                 void* ws, size_t ws_bytes, pis_stream_t stream) {
  PIS_CHECK_ARG(x && dz && dw_krsc && B > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0,
                "pis_conv3x3_wgrad: bad arguments");
  PIS_CHECK_ARG(ws_bytes >= pis_conv3x3_wgrad_ws(B, H, W, Cin, Cout),
                "pis_conv3x3_wgrad: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int acc = flags & PIS_ACCUMULATE;
  const int P = B * H * W;
  int rc;
  if (Cin == 1) {
    PIS_CHECK_ARG(Cout <= 256, "pis_conv3x3_wgrad: Cin==1 path supports Cout<=256");
    int splits, pps;
    c1_part_bytes(P, Cout, splits, pps);
    hipLaunchKernelGGL(wgrad_c1_kernel, dim3(splits), dim3(256), 0, s, x, ldx, dz, ldz, B, H, W,
                       Cout, pps, (float*)ws);
    rc = launch_status("wgrad_c1");
    if (!rc) rc = reduce_slabs((float*)ws, splits, (int64_t)Cout * 9, dw_krsc, acc, s);
  } else {
    PIS_CHECK_ARG(Cin % 64 == 0 && Cout % 64 == 0, "pis_conv3x3_wgrad: Cin/Cout must be multiples of 64");
    PIS_CHECK_ARG(ldx % 4 == 0 && ldz % 4 == 0, "pis_conv3x3_wgrad: ld must be multiples of 4");
    WgradPlan pl = plan_wgrad(Cout, 9 * Cin, P, Cout, Cin);
    WgradArgs a{};
    a.a = dz; a.lda = ldz; a.a_up2 = 0; a.Ca = Cout;
    a.b = x; a.ldb = ldx; a.b_conv3 = 1; a.Cb = Cin;
    a.B = B; a.H = H; a.W = W; a.P = P; a.Mp = Cout; a.Np = 9 * Cin; a.part = (float*)ws;
    rc = run_wgrad(a, pl, dw_krsc, acc, s);
  }
  if (rc || !db) return rc;
  return colsum(dz, ldz, P, Cout, db, acc, ws, ws_bytes, s);
}

extern "C" size_t pis_convt2x2_wgrad_ws(int B, int H, int W, int Cin, int Cout) {
  const int P = B * H * W;
  const size_t wbytes = plan_wgrad(4 * Cout, Cin, P, Cout, Cin).part_bytes;
  return std::max(wbytes, colsum_ws((int64_t)4 * P, Cout)) + 256;
}

extern "C" int pis_convt2x2_wgrad(const float* x, int ldx, const float* dy, int lddy, float* dw_ijoc,
                                  float* db, int B, int H, int W, int Cin, int Cout, int flags,
                                  void* ws, size_t ws_bytes, pis_stream_t stream) {
  PIS_CHECK_ARG(x && dy && dw_ijoc && B > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0,
                "pis_convt2x2_wgrad: bad arguments");
  PIS_CHECK_ARG(Cin % 64 == 0 && Cout % 64 == 0, "pis_convt2x2_wgrad: Cin/Cout must be multiples of 64");
  PIS_CHECK_ARG(ldx % 4 == 0 && lddy % 4 == 0, "pis_convt2x2_wgrad: ld must be multiples of 4");
  PIS_CHECK_ARG(ws_bytes >= pis_convt2x2_wgrad_ws(B, H, W, Cin, Cout),
                "pis_convt2x2_wgrad: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int acc = flags & PIS_ACCUMULATE;
  const int P = B * H * W;
  WgradPlan pl = plan_wgrad(4 * Cout, Cin, P, Cout, Cin);
  WgradArgs a{};
  a.a = dy; a.lda = lddy; a.a_up2 = 1; a.Ca = Cout;
  a.b = x; a.ldb = ldx; a.b_conv3 = 0; a.Cb = Cin;
  a.B = B; a.H = H; a.W = W; a.P = P; a.Mp = 4 * Cout; a.Np = Cin; a.part = (float*)ws;
  int rc = run_wgrad(a, pl, dw_ijoc, acc, s);
  if (rc || !db) return rc;
  return colsum(dy, lddy, (int64_t)4 * P, Cout, db, acc, ws, ws_bytes, s);
}
