// Implicit-GEMM fp32 MFMA kernels (gfx950, v_mfma_f32_32x32x2_f32) for the
// U-Net contractions of src/unet.py: 3x3 conv forward / input-gradient and
// 2x2-stride-2 transposed-conv forward / input-gradient.
//
//   C[m][n] = sum_k A[m][k] * Bt[n][k]      m = output pixel (NHWC row),
//                                            n = output channel,
//                                            k = (tap, source channel)
//
// A is gathered on the fly from an NHWC source (zero padding outside the
// image), Bt is the K-contiguous weight operand. Tiles are staged through LDS
// (register-staged double buffer, one barrier per K-step) and read back as
// 16-byte rows: lane (i, h) of a wave supplies A[i][k] for k = 8g + 4h + t,
// t = 0..3, i.e. one ds_read_b128 feeds four MFMAs (the k-permutation is
// applied identically to A and Bt, so the sum is unchanged).
#include "igemm.h"

namespace pis {

__device__ __forceinline__ void tap_offset(int mode, int t, int& dr, int& ds, int& st) {
  if (mode == TAP_CONV3) { dr = t / 3 - 1; ds = t % 3 - 1; st = 1; }
  else if (mode == TAP_UP2) { dr = t >> 1; ds = t & 1; st = 2; }
  else { dr = 0; ds = 0; st = 1; }
}

// T2D: the 128 rows of an M tile are an 8 x 16 pixel window of one image
// (needs H % 8 == 0, W % 16 == 0), so pixel coordinates are shifts, not divisions.
template <int BM, int BN, int BK, bool T2D>
__global__ __launch_bounds__(256) void igemm_f32_kernel(IGemmArgs g) {
  if (blockIdx.y) {  // batched launch (Winograd's 16 independent GEMMs): per-batch base offsets
    g.src += blockIdx.y * g.bs_src;
    g.wt += blockIdx.y * g.bs_wt;
    g.dst += blockIdx.y * g.bs_dst;
  }
  // row pitch BK+4 floats (80 or 144 bytes): 16 rows land on 16 distinct 16-B slots -> conflict-free ds_read_b128
  constexpr int LDS_ROW = BK + 4;
  constexpr int CPR = BK / 4;                           // float4 chunks per staged row
  constexpr int TM = BM / 64, TN = BN / 64;             // 32x32 tiles per wave (2x2 waves)
  constexpr int AL = BM * CPR / 256, BL = BN * CPR / 256;  // float4 staging loads per thread
  static_assert(!T2D || BM == 128, "2-D tiles are 8 x 16 pixels");
  __shared__ __attribute__((aligned(16))) float sA[2][BM * LDS_ROW];
  __shared__ __attribute__((aligned(16))) float sB[2][BN * LDS_ROW];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntn = (g.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid / ntn) * BM, n0 = (bid % ntn) * BN;
  int tb = 0, th0 = 0, tw0 = 0;
  if (T2D) {
    const int tile = bid / ntn, tpr = g.W / 16, tpi = (g.H / 8) * tpr;
    tb = tile / tpi;
    const int trem = tile - tb * tpi;
    th0 = (trem / tpr) * 8;
    tw0 = (trem % tpr) * 16;
  }

  // per-thread staging rows (fixed over the K loop)
  int a_b[AL], a_h[AL], a_w[AL];
  bool a_ok[AL];
  const int HW = g.H * g.W;
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int row = (tid + i * 256) / CPR;
    if (T2D) {
      a_ok[i] = true;
      a_b[i] = tb;
      a_h[i] = th0 + (row >> 4);
      a_w[i] = tw0 + (row & 15);
      continue;
    }
    const int m = m0 + row;
    a_ok[i] = m < g.M;
    const int mm = a_ok[i] ? m : 0;
    a_b[i] = mm / HW;
    const int rem = mm - a_b[i] * HW;
    a_h[i] = rem / g.W;
    a_w[i] = rem - a_h[i] * g.W;
  }
  const int q4 = (tid % CPR) * 4;  // channel offset inside the BK chunk

  const int nchunks = (g.Csrc + BK - 1) / BK;
  const int KT = g.ntaps * nchunks;

  f32x4 ra[AL], rb[BL];
  const bool noload = g.flags & PIS_DEBUG_NOLOAD;  // timing-only: LDS + MFMA ceiling of this loop
  auto gload = [&](int kt) {
    if (noload && kt > 0) return;
    const int tap = kt / nchunks;
    const int c = (kt - tap * nchunks) * BK + q4;
    int dr, dsh, st;
    tap_offset(g.tap_mode, tap, dr, dsh, st);
    const bool cok = c < g.Csrc;
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int hs = a_h[i] * st + dr, ws = a_w[i] * st + dsh;
      const bool ok = a_ok[i] && cok && hs >= 0 && hs < g.Hs && ws >= 0 && ws < g.Ws;
      ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (ok) {
        const size_t pix = ((size_t)a_b[i] * g.Hs + hs) * g.Ws + ws;
        ra[i] = *reinterpret_cast<const f32x4*>(g.src + pix * g.lds + c);
      }
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int n = n0 + (tid + i * 256) / CPR;
      rb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (n < g.N && cok)
        rb[i] = *reinterpret_cast<const f32x4*>(g.wt + (size_t)n * g.ldw + tap * g.Csrc + c);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int row = (tid + i * 256) / CPR;
      *reinterpret_cast<f32x4*>(&sA[buf][row * LDS_ROW + q4]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int row = (tid + i * 256) / CPR;
      *reinterpret_cast<f32x4*>(&sB[buf][row * LDS_ROW + q4]) = rb[i];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  gload(0);
  lstore(0);
  __syncthreads();
  const int li = lane & 31, lh = lane >> 5;
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) gload(kt + 1);
    const float* As = sA[cur];
    const float* Bs = sB[cur];
#pragma unroll
    for (int gg = 0; gg < BK / 8; ++gg) {
      f32x4 af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a)
        af[a] = *reinterpret_cast<const f32x4*>(
            &As[(wm * (BM / 2) + a * 32 + li) * LDS_ROW + 8 * gg + 4 * lh]);
#pragma unroll
      for (int b = 0; b < TN; ++b)
        bf[b] = *reinterpret_cast<const f32x4*>(
            &Bs[(wn * (BN / 2) + b * 32 + li) * LDS_ROW + 8 * gg + 4 * lh]);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a][t], bf[b][t], acc[a][b], 0, 0, 0);
    }
    if (kt + 1 < KT) lstore(cur ^ 1);
    __syncthreads();
  }

  // epilogue: lane owns column n = ... + li, rows i = (r&3) + 8(r>>2) + 4 lh
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int n = n0 + wn * (BN / 2) + b * 32 + li;
    if (n >= g.N) continue;
    float bias_n = 0.f;
    int o = n, ij = 0;
    if (g.epi == EPI_SCATTER2) { ij = n / g.cout_t; o = n - ij * g.cout_t; }
    if (g.bias) bias_n = g.bias[o];
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ridx = wm * (BM / 2) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        int m, bb, h, w;
        if (T2D) {
          bb = tb;
          h = th0 + (ridx >> 4);
          w = tw0 + (ridx & 15);
          m = (bb * g.H + h) * g.W + w;
        } else {
          m = m0 + ridx;
          if (m >= g.M) continue;
          bb = m / HW;
          const int rem = m - bb * HW;
          h = rem / g.W;
          w = rem - h * g.W;
        }
        float v = acc[a][b][r] + bias_n;
        if (g.flags & PIS_RELU) v = fmaxf(v, 0.f);
        if (g.flags & PIS_MASK) v = (g.mask[(size_t)m * g.ldm + n] > 0.f) ? v : 0.f;
        if (g.flags & PIS_SCALE) v *= g.scale[(size_t)bb * g.N + n];
        size_t off;
        if (g.epi == EPI_SCATTER2) {
          const int oh = 2 * h + (ij >> 1), ow = 2 * w + (ij & 1);
          off = (((size_t)bb * 2 * g.H + oh) * (2 * g.W) + ow) * g.ldd + o;
        } else {
          off = (size_t)m * g.ldd + n;
        }
        if (g.flags & PIS_ACCUMULATE) v += g.dst[off];
        g.dst[off] = v;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// 3x3 conv (fwd, or dgrad on flipped weights) from a staged input halo.
//
// Block tile: 128 output pixels = an 8-row x 16-column window of one image,
// x BN output channels; 2x2 waves, 64 px x BN/2 channels each. The K loop walks
// CK-channel slices of the input: per stage the block stages the 10x18-pixel
// input halo of the window and the weights of all 9 taps once, then every tap
// reads its shifted window from LDS (9 * CK/2 * TN * 2 MFMAs per wave per
// barrier), so each input element is fetched once per block instead of once
// per tap. Both LDS images split the slice into two halves by MFMA lane half:
// X[h][pixel][CK/2], W[tap][h][n][CK/2]; lane half h supplies channel
// h*CK/2 + s to MFMA s of the slice for both operands, so the sum is unchanged
// and every fragment is one contiguous 8- or 16-byte read per lane.
// ---------------------------------------------------------------------------
template <int BN, int CK>
__global__ __launch_bounds__(256, (BN >= 256 ? 2 : 1)) void conv3x3_halo_kernel(IGemmArgs g) {
  constexpr int TR = 8, TC = 16, HR = TR + 2, HC = TC + 2, HP = HR * HC;  // 180 halo pixels
  constexpr int TM = 2, TN = BN / 64, HK = CK / 2;  // HK channels per lane half
  constexpr int XF4 = HP * CK / 4, WF4 = 9 * BN * CK / 4;  // float4 per stage
  constexpr int XL = (XF4 + 255) / 256, WL = (WF4 + 255) / 256;
  typedef float hvec __attribute__((ext_vector_type(HK)));
  __shared__ __attribute__((aligned(16))) float sX[2][HP * CK];
  __shared__ __attribute__((aligned(16))) float sW[2][9 * BN * CK];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int li = lane & 31, lh = lane >> 5;
  const int ntn = (g.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid / ntn, n0 = (bid % ntn) * BN;
  const int tpr = g.W / TC, tpi = (g.H / TR) * tpr;  // tiles per tile-row, per image
  const int b = tile / tpi, trem = tile - b * tpi;
  const int h0 = (trem / tpr) * TR, w0 = (trem % tpr) * TC;
  const int nchunks = g.Csrc / CK;

  f32x4 rx[XL], rw[WL];
  const bool noload = g.flags & PIS_DEBUG_NOLOAD;  // timing-only: LDS + MFMA ceiling of this loop
  auto gload = [&](int kc) {
    if (noload && kc > 0) return;
    const int c = kc * CK;
#pragma unroll
    for (int i = 0; i < XL; ++i) {
      const int idx = tid + i * 256;  // (pixel, 4-channel chunk)
      const int px = idx / (CK / 4), q = idx - px * (CK / 4);
      const int hs = h0 + px / HC - 1, ws = w0 + px % HC - 1;
      rx[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (idx < XF4 && hs >= 0 && hs < g.H && ws >= 0 && ws < g.W)
        rx[i] = *reinterpret_cast<const f32x4*>(g.src + (((size_t)b * g.H + hs) * g.W + ws) * g.lds + c + 4 * q);
    }
#pragma unroll
    for (int i = 0; i < WL; ++i) {
      const int idx = tid + i * 256;  // (tap, n, 4-channel chunk)
      const int q = idx % (CK / 4), tn = idx / (CK / 4);
      const int t = tn / BN, nl = tn - t * BN;
      rw[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (idx < WF4 && n0 + nl < g.N)
        rw[i] = *reinterpret_cast<const f32x4*>(g.wt + (size_t)(n0 + nl) * g.ldw + t * g.Csrc + c + 4 * q);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < XL; ++i) {
      const int idx = tid + i * 256;
      if (idx >= XF4) continue;
      const int px = idx / (CK / 4), q = idx - px * (CK / 4);
      float* X = sX[buf];
      if (CK == 4) {
        *reinterpret_cast<float2*>(&X[(0 * HP + px) * 2]) = make_float2(rx[i][0], rx[i][1]);
        *reinterpret_cast<float2*>(&X[(1 * HP + px) * 2]) = make_float2(rx[i][2], rx[i][3]);
      } else {  // CK == 8: chunk q is lane half q
        *reinterpret_cast<f32x4*>(&X[(q * HP + px) * 4]) = rx[i];
      }
    }
#pragma unroll
    for (int i = 0; i < WL; ++i) {
      const int idx = tid + i * 256;
      if (idx >= WF4) continue;
      const int q = idx % (CK / 4), tn = idx / (CK / 4);
      const int t = tn / BN, nl = tn - t * BN;
      float* Wt = sW[buf];
      if (CK == 4) {
        *reinterpret_cast<float2*>(&Wt[((t * 2 + 0) * BN + nl) * 2]) = make_float2(rw[i][0], rw[i][1]);
        *reinterpret_cast<float2*>(&Wt[((t * 2 + 1) * BN + nl) * 2]) = make_float2(rw[i][2], rw[i][3]);
      } else {
        *reinterpret_cast<f32x4*>(&Wt[((t * 2 + q) * BN + nl) * 4]) = rw[i];
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int c = 0; c < TN; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;

  // this lane's output pixels (rows of its two 32-row MFMA tiles) in halo coordinates
  int pbase[TM];
#pragma unroll
  for (int a = 0; a < TM; ++a) {
    const int idx = wm * 64 + a * 32 + li;
    pbase[a] = (idx / TC) * HC + (idx % TC);
  }

  gload(0);
  lstore(0);
  __syncthreads();
  for (int kc = 0; kc < nchunks; ++kc) {
    const int cur = kc & 1;
    if (kc + 1 < nchunks) gload(kc + 1);
    const float* X = sX[cur] + lh * HP * HK;
    const float* Wt = sW[cur];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int toff = (t / 3) * HC + (t % 3);
      hvec af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a] = *reinterpret_cast<const hvec*>(&X[(pbase[a] + toff) * HK]);
#pragma unroll
      for (int c = 0; c < TN; ++c)
        bf[c] = *reinterpret_cast<const hvec*>(&Wt[((t * 2 + lh) * BN + wn * (BN / 2) + c * 32 + li) * HK]);
#pragma unroll
      for (int s = 0; s < HK; ++s)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int c = 0; c < TN; ++c)
            acc[a][c] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a][s], bf[c][s], acc[a][c], 0, 0, 0);
    }
    if (kc + 1 < nchunks) lstore(cur ^ 1);
    __syncthreads();
  }

  const int HWimg = g.H * g.W;
#pragma unroll
  for (int c = 0; c < TN; ++c) {
    const int n = n0 + wn * (BN / 2) + c * 32 + li;
    if (n >= g.N) continue;
    const float bias_n = g.bias ? g.bias[n] : 0.f;
    const float sc = (g.flags & PIS_SCALE) ? g.scale[(size_t)b * g.N + n] : 1.f;
#pragma unroll
    for (int a = 0; a < TM; ++a) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int idx = wm * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        const size_t m = (size_t)b * HWimg + (size_t)(h0 + idx / TC) * g.W + w0 + idx % TC;
        float v = acc[a][c][r] + bias_n;
        if (g.flags & PIS_RELU) v = fmaxf(v, 0.f);
        if (g.flags & PIS_MASK) v = (g.mask[m * g.ldm + n] > 0.f) ? v : 0.f;
        v *= sc;
        const size_t off = m * g.ldd + n;
        if (g.flags & PIS_ACCUMULATE) v += g.dst[off];
        g.dst[off] = v;
      }
    }
  }
}

static bool halo_ok(const IGemmArgs& a) {
  return a.tap_mode == TAP_CONV3 && a.epi == EPI_NHWC && a.W % 16 == 0 && a.H % 8 == 0 &&
         a.Csrc % 4 == 0 && a.lds % 4 == 0 && a.ldw % 4 == 0;
}


int launch_igemm(const IGemmArgs& a, hipStream_t s, int batches) {
  // tile choice: BN=64 for narrow outputs, BM=128; K-step from the tuning table
  const int ntm = (int)cdiv(a.M, 128);
  const int bk = tune_get(PIS_TUNE_IGEMM_BK);
  IGemmArgs& m = const_cast<IGemmArgs&>(a);
  if (tune_get(PIS_TUNE_DEBUG_NOLOAD)) m.flags |= PIS_DEBUG_NOLOAD;
  const bool t2d = a.W % 16 == 0 && a.H % 8 == 0 && bk != 32;
  if (a.N <= 64) {
    const int grid = ntm * (int)cdiv(a.N, 64);
    if (bk == 32)
      hipLaunchKernelGGL((igemm_f32_kernel<128, 64, 32, false>), dim3(grid, batches), dim3(256), 0, s, a);
    else if (t2d)
      hipLaunchKernelGGL((igemm_f32_kernel<128, 64, 16, true>), dim3(grid, batches), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((igemm_f32_kernel<128, 64, 16, false>), dim3(grid, batches), dim3(256), 0, s, a);
  } else {
    const int grid = ntm * (int)cdiv(a.N, 128);
    if (bk == 32)
      hipLaunchKernelGGL((igemm_f32_kernel<128, 128, 32, false>), dim3(grid, batches), dim3(256), 0, s, a);
    else if (t2d)
      hipLaunchKernelGGL((igemm_f32_kernel<128, 128, 16, true>), dim3(grid, batches), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((igemm_f32_kernel<128, 128, 16, false>), dim3(grid, batches), dim3(256), 0, s, a);
  }
  return launch_status("igemm_f32");
}

int launch_conv3x3(const IGemmArgs& a, hipStream_t s) {
  if (!halo_ok(a) || !tune_get(PIS_TUNE_CONV_HALO)) return launch_igemm(a, s);
  if (tune_get(PIS_TUNE_DEBUG_NOLOAD)) const_cast<IGemmArgs&>(a).flags |= PIS_DEBUG_NOLOAD;
  const int tiles = (a.M / (8 * 16));
  const int variant = tune_get(PIS_TUNE_HALO_VARIANT);
  const double flop = 2.0 * a.M * a.N * 9.0 * a.Csrc;
  launch_hook("conv3x3_halo", 0, s, flop);
  if (a.N <= 64) {
    // 8-channel slices measured faster for the forward convs, 4-channel slices for
    // the masked dgrad epilogue (tools/bench_kernels.py --key 4 --variants 0,1,3)
    const bool ck4 = variant == 1 || (variant == 0 && (a.flags & PIS_MASK));
    if (ck4 || a.Csrc % 8 != 0)
      hipLaunchKernelGGL((conv3x3_halo_kernel<64, 4>), dim3(tiles * (int)cdiv(a.N, 64)), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((conv3x3_halo_kernel<64, 8>), dim3(tiles * (int)cdiv(a.N, 64)), dim3(256), 0, s, a);
  } else if (a.N >= 256 && variant == 2) {
    hipLaunchKernelGGL((conv3x3_halo_kernel<256, 4>), dim3(tiles * (int)cdiv(a.N, 256)), dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL((conv3x3_halo_kernel<128, 4>), dim3(tiles * (int)cdiv(a.N, 128)), dim3(256), 0, s, a);
  }
  launch_hook("conv3x3_halo", 1, s, flop);
  return launch_status("conv3x3_halo");
}

// Cin == 1, Cout == 64, W % 64 == 0: block = one 64-pixel segment of R image rows; the
// (R + 2) x 66 input window is staged in LDS once, thread (pixel group pg = t / 16, channel quad
// t % 16) computes pixels pg + 16 k (k < 4) of each row and every wave stores 4 whole pixels (1 KB)
// per instruction (no per-pixel index divisions, no redundant x loads). R rows per block amortise
// the 36 weight loads per thread (R = 4 when H % 4 == 0).
template <int R>
__global__ __launch_bounds__(256) void conv3x3_c1_row_kernel(const float* __restrict__ x, int ldx,
                                                             const float* __restrict__ w,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ scale,
                                                             float* __restrict__ y, int ldy, int H, int W,
                                                             int flags) {
  constexpr int Cout = 64, SEG = 64;
  __shared__ float xs[R + 2][SEG + 2];
  const int segs = W / SEG, hb = H / R;
  const int bh = blockIdx.x / segs, w0 = (blockIdx.x - bh * segs) * SEG;
  const int b = bh / hb, h0 = (bh - b * hb) * R;
  const int tid = threadIdx.x;
  for (int i = tid; i < (R + 2) * (SEG + 2); i += 256) {
    const int r = i / (SEG + 2), c = i - r * (SEG + 2);
    const int hh = h0 + r - 1, ww = w0 + c - 1;
    xs[r][c] = (hh >= 0 && hh < H && ww >= 0 && ww < W) ? x[(((size_t)b * H + hh) * W + ww) * ldx] : 0.f;
  }
  const int c4 = (tid & 15) * 4, pg = tid >> 4;
  f32x4 wt[9], b4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    b4[j] = bias ? bias[c4 + j] : 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) wt[t][j] = w[(c4 + j) * 9 + t];
  }
  f32x4 sc = {1.f, 1.f, 1.f, 1.f};
  if (flags & PIS_SCALE) sc = *reinterpret_cast<const f32x4*>(scale + (size_t)b * Cout + c4);
  __syncthreads();
#pragma unroll
  for (int rr = 0; rr < R; ++rr) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int px = pg + 16 * k;
      f32x4 acc = b4;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const float xv = xs[rr + t / 3][px + t % 3];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = fmaf(xv, wt[t][j], acc[j]);
      }
      if (flags & PIS_RELU) {
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = fmaxf(acc[j], 0.f);
      }
      acc *= sc;
      *reinterpret_cast<f32x4*>(y + (((size_t)b * H + h0 + rr) * W + w0 + px) * ldy + c4) = acc;
    }
  }
}

__global__ __launch_bounds__(256) void conv3x3_c1_fwd_kernel(const float* __restrict__ x, int ldx,
                                                             const float* __restrict__ w,
                                                             const float* __restrict__ bias,
                                                             const float* __restrict__ scale,
                                                             float* __restrict__ y, int ldy, int B, int H,
                                                             int W, int Cout, int flags) {
  // Cin == 1 (enc1.conv0): an HBM-write-bound stream (4*Cout B per pixel). Cout/4 lanes per
  // pixel, each owning 4 output channels whose 9 taps + bias live in registers; the grid
  // strides over pixels so the weights are loaded once per thread.
  const int lanes_per_pix = Cout / 4;
  const int pix_per_block = 256 / lanes_per_pix;
  const int lp = threadIdx.x / lanes_per_pix;
  const int c4 = (threadIdx.x - lp * lanes_per_pix) * 4;
  if (lp >= pix_per_block) return;
  f32x4 wt[9], b4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    b4[j] = bias ? bias[c4 + j] : 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) wt[t][j] = w[(c4 + j) * 9 + t];
  }
  const int HW = H * W;
  const int64_t npix = (int64_t)B * HW;
  for (int64_t p = (int64_t)blockIdx.x * pix_per_block + lp; p < npix; p += (int64_t)gridDim.x * pix_per_block) {
    const int b = (int)(p / HW), rem = (int)(p - (int64_t)b * HW), h = rem / W, wc = rem - h * W;
    const float* xb = x + (int64_t)b * HW * ldx;
    f32x4 acc = b4;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int hh = h + t / 3 - 1, ww = wc + t % 3 - 1;
      const float xv = (hh >= 0 && hh < H && ww >= 0 && ww < W) ? xb[(int64_t)(hh * W + ww) * ldx] : 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = fmaf(xv, wt[t][j], acc[j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float v = acc[j];
      if (flags & PIS_RELU) v = fmaxf(v, 0.f);
      if (flags & PIS_SCALE) v *= scale[(size_t)b * Cout + c4 + j];
      acc[j] = v;
    }
    *reinterpret_cast<f32x4*>(y + p * ldy + c4) = acc;
  }
}

__global__ void conv3x3_flip_kernel(const float* __restrict__ w, float* __restrict__ wf, int Cin,
                                    int Cout) {
  const int64_t n_el = (int64_t)Cin * 9 * Cout;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_el;
       i += (int64_t)gridDim.x * blockDim.x) {
    // destination index i = ((c*3 + r)*3 + s)*Cout + n
    const int n = (int)(i % Cout);
    const int64_t rest = i / Cout;
    const int rs = (int)(rest % 9);
    const int c = (int)(rest / 9);
    const int r = rs / 3, s = rs % 3;
    wf[i] = w[(((int64_t)n * 3 + (2 - r)) * 3 + (2 - s)) * Cin + c];
  }
}

__global__ void convt_prep_kernel(const float* __restrict__ w, float* __restrict__ wc, int Cin,
                                  int Cout) {
  // w[i][j][o][c] -> wc[c][i][j][o]
  const int64_t n_el = (int64_t)4 * Cout * Cin;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n_el;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int o = (int)(e % Cout);
    const int64_t rest = e / Cout;
    const int ij = (int)(rest % 4);
    const int c = (int)(rest / 4);
    wc[e] = w[((int64_t)ij * Cout + o) * Cin + c];
  }
}

}  // namespace pis

using namespace pis;

// Winograd policy (winograd.hip): where its GEMMs stay MFMA-bound and beat the direct kernels
static bool wino_wanted_dims(int H, int W, int C, int N) {
  const int mode = tune_get(PIS_TUNE_WINOGRAD);
  if (mode == 0 || H % 2 || W % 2 || C % 4 || N % 4) return false;
  if (mode == 2) return true;
  // measured (tools/bench_kernels.py --key 8 --variants 1,2 --ops fwd,dgrad, B=8):
  // F(4x4,3x3) beats the direct halo kernels from 128 channels on either side (dec1.conv0
  // fwd -22 %, dgrad -27 %; enc2.conv1 -41 %) and only loses at 64 -> 64 (+1.5-3 %);
  // F(2x2,3x3) needs >= 256 contraction channels and 128 outputs. With the bf16x6 GEMMs
  // (key 10 = 3) F(4x4,3x3) also wins at 64 -> 64 (enc1.conv1 fwd -13 %, dgrad -11 %).
  if (wino_tile(H, W) == 4)
    return C >= 128 || N >= 128 || (tune_get(PIS_TUNE_WINO_TILE) >= 3 && C >= 64 && N >= 64);
  return C >= 256 && N >= 128;
}

namespace pis {
bool wino_fused_wanted(int B, int H, int W, int C, int N);  // winograd.hip
}

// F(6x6,3x3) for a layer's forward and input gradient (pis_tune key 47; csrc/winograd.hip
// launch_wino6): both directions on the batched fp16x3 GEMM (Winograd-wanted, neither direct nor
// fused), 64-aligned channels, an F(4x4)-capable grid (the weight gradient keeps F(3x3,4x4)), and
// at least 10 % fewer products on the ragged 6 x 6 tile grid: 128^2 and 64^2 at C2 (0.84 of
// F(4x4)'s), not 32^2 (ceil(32 / 6)^2 x 64 = 32^2 / 16 x 36: no gain)
bool pis::wino6_layer(int B, int H, int W, int Cin, int Cout) {
  if (tune_get(PIS_TUNE_WINO_F6) == 0 || tune_get(PIS_TUNE_WINO_TILE) != 4 || B <= 0) return false;
  if (wino_tile(H, W) != 4 || Cin % 64 || Cout % 64) return false;
  if (direct_h3_wanted(H, W, Cin, Cout, 4) || direct_h3_wanted(H, W, Cout, Cin, 4)) return false;
  if (!wino_wanted_dims(H, W, Cin, Cout) || !wino_wanted_dims(H, W, Cout, Cin)) return false;
  if (wino_fused_wanted(B, H, W, Cin, Cout) || wino_fused_wanted(B, H, W, Cout, Cin)) return false;
  const int64_t p6 = (int64_t)64 * ((H + 5) / 6) * ((W + 5) / 6), p4 = (int64_t)36 * (H / 4) * (W / 4);
  return 10 * p6 <= 9 * p4;
}

static int dispatch_conv3x3(const IGemmArgs& a, int B, void* ws, size_t ws_bytes, hipStream_t s,
                            float* keep_v = nullptr, bool v_ready = false) {
  // the direct fp16x3 kernel (pis_tune key 29) where its policy takes the layer; a kept forward
  // transform is then still owed to the layer's Winograd weight gradient
  // (PIS_FILTER_READY here: a.wt is the layer's split from pis_conv3x3_filter(s), format 3)
  if (ws && !v_ready && a.tap_mode == TAP_CONV3 && a.epi == EPI_NHWC &&
      direct_h3_wanted(a.H, a.W, a.Csrc, a.N, a.lds) &&
      (a.filter_ready || ws_bytes >= direct_h3_ws_bytes(a.Csrc, a.N))) {
    int rc = launch_direct_h3(a, B, ws, ws_bytes, s, a.w_unflipped != 0, a.filter_ready);
    if (!rc && keep_v) rc = launch_wino_input(a.src, a.lds, B, a.H, a.W, a.Csrc, keep_v, s, 4);
    return rc;
  }
  // a kept transform is computed either way: then Winograd wins even where the plain policy
  // prefers the direct kernel (64 -> 64 at 512^2: +2 % forward, -27 % weight gradient)
  if (ws && wino_ok(a) && (keep_v || wino_wanted_dims(a.H, a.W, a.Csrc, a.N)) &&
      ws_bytes >= wino_ws_bytes(B, a.H, a.W, a.Csrc, a.N))
    return launch_wino3x3(a, B, ws, s, keep_v, v_ready);
  if (a.filter_ready) {
    set_error("conv3x3: PIS_FILTER_READY but this call does not take the F(4x4,3x3) path");
    return PIS_ERR_ARG;
  }
  if (v_ready) {
    set_error("pis_conv3x3_dgrad_ex: PIS_WINO_PREPARED but this call does not take the Winograd path");
    return PIS_ERR_ARG;
  }
  int rc = launch_conv3x3(a, s);
  // direct path taken (e.g. a small workspace): the kept transform is still owed to the wgrad
  if (!rc && keep_v) rc = launch_wino_input(a.src, a.lds, B, a.H, a.W, a.Csrc, keep_v, s, 4);
  return rc;
}

size_t wino_wgrad_keep_bytes(int B, int H, int W, int Cin, int Cout);  // wgrad.hip

extern "C" size_t pis_conv3x3_ex_ws(int B, int H, int W, int Cin, int Cout) {
  size_t need = 0;
  if (direct_h3_wanted(H, W, Cin, Cout, 4)) need = std::max(need, direct_h3_ws_bytes(Cin, Cout));
  if (direct_h3_wanted(H, W, Cout, Cin, 4)) need = std::max(need, direct_h3_ws_bytes(Cout, Cin));
  const bool keepable = Cin % 4 == 0 && wino_tile(H, W) == 4 && wino_wgrad_keep_bytes(B, H, W, Cin, Cout) > 0;
  if (keepable || wino_wanted_dims(H, W, Cin, Cout)) need = std::max(need, wino_ws_bytes(B, H, W, Cin, Cout));  // fwd
  if (wino_wanted_dims(H, W, Cout, Cin)) need = std::max(need, wino_ws_bytes(B, H, W, Cout, Cin));  // dgrad
  return need;
}

extern "C" int pis_conv3x3_fwd(const float* x, int ldx, const float* w_krsc, const float* bias,
                               const float* scale, float* y, int ldy, int B, int H, int W, int Cin,
                               int Cout, int flags, pis_stream_t stream) {
  return pis_conv3x3_fwd_ex(x, ldx, w_krsc, bias, scale, y, ldy, B, H, W, Cin, Cout, flags, nullptr, 0, stream);
}

extern "C" size_t pis_conv3x3_keep_bytes(int B, int H, int W, int Cin, int Cout) {
  if (Cin % 4 || wino_tile(H, W) != 4 || tune_get(PIS_TUNE_WINOGRAD) == 0) return 0;
  if (wino6_layer(B, H, W, Cin, Cout)) return 0;  // F(6x6) forward: the weight gradient transforms x itself
  return wino_wgrad_keep_bytes(B, H, W, Cin, Cout);
}

extern "C" int pis_conv3x3_fwd_keep(const float* x, int ldx, const float* w_krsc, const float* bias,
                                    const float* scale, float* y, int ldy, int B, int H, int W, int Cin,
                                    int Cout, int flags, void* ws, size_t ws_bytes, float* keep,
                                    pis_stream_t stream) {
  const size_t kb = pis_conv3x3_keep_bytes(B, H, W, Cin, Cout);
  if (!keep || kb == 0)
    return pis_conv3x3_fwd_ex(x, ldx, w_krsc, bias, scale, y, ldy, B, H, W, Cin, Cout, flags, ws, ws_bytes, stream);
  PIS_CHECK_ARG(x && w_krsc && y && B > 0 && ldx % 4 == 0 && ldy % 4 == 0 && Cout % 4 == 0,
                "pis_conv3x3_fwd_keep: bad arguments");
  PIS_CHECK_ARG(!(flags & PIS_SCALE) || scale, "pis_conv3x3_fwd_keep: PIS_SCALE without scale");
  IGemmArgs a{};
  a.src = x; a.lds = ldx; a.Hs = H; a.Ws = W; a.H = H; a.W = W; a.M = B * H * W;
  a.Csrc = Cin; a.ntaps = 9; a.tap_mode = TAP_CONV3; a.wt = w_krsc; a.ldw = 9 * Cin; a.N = Cout;
  a.epi = EPI_NHWC; a.bias = bias; a.scale = scale; a.dst = y; a.ldd = ldy;
  a.flags = flags & (PIS_RELU | PIS_SCALE | PIS_ACCUMULATE);
  a.filter_ready = (flags & PIS_FILTER_READY) != 0;
  return dispatch_conv3x3(a, B, ws, ws_bytes, (hipStream_t)stream, keep);
}

extern "C" int pis_conv3x3_fwd_pool(const float* x, int ldx, const float* w_krsc, const float* bias,
                                    const float* scale, float* y, int ldy, int B, int H, int W, int Cin,
                                    int Cout, int flags, void* ws, size_t ws_bytes, float* keep, float* pool,
                                    pis_stream_t stream) {
  PIS_CHECK_ARG(pool && H % 2 == 0 && W % 2 == 0 && !(flags & PIS_ACCUMULATE),
                "pis_conv3x3_fwd_pool: needs a pool buffer, even H and W, no PIS_ACCUMULATE");
  PIS_CHECK_ARG(x && w_krsc && y && B > 0 && Cin > 0 && (Cin == 1 || ldx % 4 == 0) && ldy % 4 == 0 &&
                    Cout % 4 == 0,
                "pis_conv3x3_fwd_pool: bad arguments");
  PIS_CHECK_ARG(!(flags & PIS_SCALE) || scale, "pis_conv3x3_fwd_pool: PIS_SCALE without scale");
  const bool kept = keep && pis_conv3x3_keep_bytes(B, H, W, Cin, Cout) > 0;
  IGemmArgs a{};
  a.src = x; a.lds = ldx; a.Hs = H; a.Ws = W; a.H = H; a.W = W; a.M = B * H * W;
  a.Csrc = Cin; a.ntaps = 9; a.tap_mode = TAP_CONV3; a.wt = w_krsc; a.ldw = 9 * Cin; a.N = Cout;
  a.epi = EPI_NHWC; a.bias = bias; a.scale = scale; a.dst = y; a.ldd = ldy;
  a.flags = flags & (PIS_RELU | PIS_SCALE);
  a.filter_ready = (flags & PIS_FILTER_READY) != 0;
  // the direct fp16x3 kernel and the F(4x4,3x3) output epilogues pool the tile they just wrote;
  // every other path pools after
  if (Cin > 1 && ws && direct_h3_wanted(H, W, Cin, Cout, ldx) &&
      (a.filter_ready || ws_bytes >= direct_h3_ws_bytes(Cin, Cout))) {
    a.pool = pool;
    return dispatch_conv3x3(a, B, ws, ws_bytes, (hipStream_t)stream, kept ? keep : nullptr);
  }
  if (Cin > 1 && ws && wino_ok(a) && wino_tile(H, W) == 4 && (kept || wino_wanted_dims(H, W, Cin, Cout)) &&
      ws_bytes >= wino_ws_bytes(B, H, W, Cin, Cout)) {
    a.pool = pool;
    return dispatch_conv3x3(a, B, ws, ws_bytes, (hipStream_t)stream, kept ? keep : nullptr);
  }
  int rc = pis_conv3x3_fwd_keep(x, ldx, w_krsc, bias, scale, y, ldy, B, H, W, Cin, Cout, flags, ws, ws_bytes,
                                keep, stream);
  if (rc) return rc;
  return pis_maxpool2x2_fwd(y, ldy, pool, B, H, W, Cout, stream);
}

extern "C" int pis_conv3x3_fwd_ex(const float* x, int ldx, const float* w_krsc, const float* bias,
                                  const float* scale, float* y, int ldy, int B, int H, int W, int Cin,
                                  int Cout, int flags, void* ws, size_t ws_bytes, pis_stream_t stream) {
  PIS_CHECK_ARG(x && w_krsc && y && B > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0,
                "pis_conv3x3_fwd: bad arguments");
  PIS_CHECK_ARG(!(flags & PIS_SCALE) || scale, "pis_conv3x3_fwd: PIS_SCALE without scale");
  PIS_CHECK_ARG(ldy % 4 == 0 && Cout % 4 == 0, "pis_conv3x3_fwd: ldy/Cout must be multiples of 4");
  hipStream_t s = (hipStream_t)stream;
  PIS_CHECK_ARG(!(flags & PIS_FILTER_READY) || Cin > 1, "pis_conv3x3_fwd: PIS_FILTER_READY with Cin == 1");
  if (Cin == 1 && Cout == 64 && W % 64 == 0) {
    if (H % 4 == 0)
      hipLaunchKernelGGL(conv3x3_c1_row_kernel<4>, dim3((unsigned)(B * (H / 4) * (W / 64))), dim3(256), 0, s, x, ldx,
                         w_krsc, bias, scale, y, ldy, H, W, flags);
    else
      hipLaunchKernelGGL(conv3x3_c1_row_kernel<1>, dim3((unsigned)(B * H * (W / 64))), dim3(256), 0, s, x, ldx,
                         w_krsc, bias, scale, y, ldy, H, W, flags);
    return launch_status("conv3x3_c1_row");
  }
  if (Cin == 1) {
    PIS_CHECK_ARG(Cout <= 1024, "pis_conv3x3_fwd: Cin==1 path supports Cout<=1024");
    const int64_t threads = (int64_t)B * H * W * (Cout / 4);
    const int64_t blocks = std::min<int64_t>(cdiv(threads, 256), 4096);
    hipLaunchKernelGGL(conv3x3_c1_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, s, x, ldx, w_krsc, bias,
                       scale, y, ldy, B, H, W, Cout, flags);
    return launch_status("conv3x3_c1_fwd");
  }
  PIS_CHECK_ARG(Cin % 4 == 0 && ldx % 4 == 0, "pis_conv3x3_fwd: Cin/ldx must be multiples of 4");
  IGemmArgs a{};
  a.src = x; a.lds = ldx; a.Hs = H; a.Ws = W; a.H = H; a.W = W; a.M = B * H * W;
  a.Csrc = Cin; a.ntaps = 9; a.tap_mode = TAP_CONV3; a.wt = w_krsc; a.ldw = 9 * Cin; a.N = Cout;
  a.epi = EPI_NHWC; a.bias = bias; a.scale = scale; a.dst = y; a.ldd = ldy;
  a.flags = flags & (PIS_RELU | PIS_SCALE | PIS_ACCUMULATE);
  a.filter_ready = (flags & PIS_FILTER_READY) != 0;
  return dispatch_conv3x3(a, B, ws, ws_bytes, s);
}

extern "C" int pis_conv3x3_flip(const float* w_krsc, float* w_flip, int Cin, int Cout,
                                pis_stream_t stream) {
  PIS_CHECK_ARG(w_krsc && w_flip && Cin > 0 && Cout > 0, "pis_conv3x3_flip: bad arguments");
  const int64_t n = (int64_t)Cin * 9 * Cout;
  const int grid = (int)std::min<int64_t>(cdiv(n, 256), 4096);
  hipLaunchKernelGGL(conv3x3_flip_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, w_krsc,
                     w_flip, Cin, Cout);
  return launch_status("conv3x3_flip");
}

namespace pis {  // winograd.hip
int wino_filter_format(int B, int H, int W, int C, int N, bool kept);
int launch_wino4_filter_only(const float* w, int C, int N, int dgrad, int format, void* out, hipStream_t s);
int launch_wino4_filter_batch(int n, const float* const* w, void* const* out, const int* C, const int* N,
                              const int* dgrad, const int* format, hipStream_t s);
}  // namespace pis

// the filter transform pis_conv3x3_{fwd_keep,fwd_pool,dgrad_ex} would compute (engine shapes:
// kept forward transforms, prepared 32-aligned input gradients)
static int filter_format(int B, int H, int W, int Cin, int Cout, int dgrad) {
  if (B <= 0 || H <= 0 || W <= 0 || Cin % 4 || Cout % 4 || Cin < 4) return 0;
  // 4: the F(6x6,3x3) transform U[64][N][C] (input gradient: from the ORIGINAL weights)
  if (wino6_layer(B, H, W, Cin, Cout)) return 4;
  // 3: the call takes the direct fp16x3 kernel — its "filter transform" is the weight split
  if (dgrad ? direct_h3_wanted(H, W, Cout, Cin, 4) : direct_h3_wanted(H, W, Cin, Cout, 4)) return 3;
  if (dgrad) {
    if (Cin % 32 || Cout % 32 || !wino_wanted_dims(H, W, Cout, Cin)) return 0;
    return wino_filter_format(B, H, W, Cout, Cin, false);
  }
  if (pis_conv3x3_keep_bytes(B, H, W, Cin, Cout) == 0 && !wino_wanted_dims(H, W, Cin, Cout)) return 0;
  return wino_filter_format(B, H, W, Cin, Cout, pis_conv3x3_keep_bytes(B, H, W, Cin, Cout) > 0);
}

extern "C" size_t pis_conv3x3_filter_bytes(int B, int H, int W, int Cin, int Cout, int dgrad) {
  const int f = filter_format(B, H, W, Cin, Cout, dgrad);
  if (f == 0) return 0;
  const size_t nc = (size_t)36 * Cin * Cout;
  const int C = dgrad ? Cout : Cin, N = dgrad ? Cin : Cout;  // contraction, outputs
  if (f == 3) return direct_h3_ws_bytes(C, N);
  if (f == 4) return (size_t)64 * Cin * Cout * sizeof(float);
  if (f == 2 && tune_get(PIS_TUNE_WINO_GEMM_OUT_H3) != 0)  // fp16x3: hi / lo planes + one scale per output
    return 2 * nc * sizeof(_Float16) + (size_t)N * sizeof(float);
  return f == 2 ? 3 * nc * sizeof(__bf16) : nc * sizeof(float);
}

extern "C" int pis_conv3x3_filter(const float* w, int B, int H, int W, int Cin, int Cout, int dgrad, void* out,
                                  size_t out_bytes, pis_stream_t stream) {
  const int f = filter_format(B, H, W, Cin, Cout, dgrad);
  PIS_CHECK_ARG(w && out && f != 0, "pis_conv3x3_filter: no F(4x4,3x3) GEMM path for these shapes");
  PIS_CHECK_ARG(out_bytes >= pis_conv3x3_filter_bytes(B, H, W, Cin, Cout, dgrad), "pis_conv3x3_filter: output too small");
  if (f == 3) {  // the direct kernel's split (input gradient: of the ORIGINAL weights)
    const int dg = dgrad ? 1 : 0;
    void* o = out;
    return launch_direct_wsplit_batch(1, &w, &o, &Cin, &Cout, &dg, (hipStream_t)stream);
  }
  // forward: contraction C = Cin, outputs N = Cout; input gradient: C = Cout, N = Cin
  if (f == 4)
    return dgrad ? launch_wino6_filter_only(w, Cout, Cin, 1, out, (hipStream_t)stream)
                 : launch_wino6_filter_only(w, Cin, Cout, 0, out, (hipStream_t)stream);
  return dgrad ? launch_wino4_filter_only(w, Cout, Cin, 1, f, out, (hipStream_t)stream)
               : launch_wino4_filter_only(w, Cin, Cout, 0, f, out, (hipStream_t)stream);
}

extern "C" int pis_conv3x3_filter_format(int B, int H, int W, int Cin, int Cout, int dgrad) {
  return filter_format(B, H, W, Cin, Cout, dgrad);
}

extern "C" int pis_conv3x3_filters(const pis_filter_job* jobs, int n, pis_stream_t stream) {
  PIS_CHECK_ARG(jobs && n >= 0 && n <= PIS_FILTER_MAX_JOBS, "pis_conv3x3_filters: bad arguments");
  const float* w[PIS_FILTER_MAX_JOBS];
  void* out[PIS_FILTER_MAX_JOBS];
  int C[PIS_FILTER_MAX_JOBS], N[PIS_FILTER_MAX_JOBS], dg[PIS_FILTER_MAX_JOBS], fmt[PIS_FILTER_MAX_JOBS];
  // the direct kernel's splits (format 3) go to a second launch
  const float* dw[PIS_FILTER_MAX_JOBS];
  void* dout[PIS_FILTER_MAX_JOBS];
  int dci[PIS_FILTER_MAX_JOBS], dco[PIS_FILTER_MAX_JOBS], ddg[PIS_FILTER_MAX_JOBS];
  int nw = 0, nd = 0;
  for (int k = 0; k < n; ++k) {
    const pis_filter_job& j = jobs[k];
    const int f = filter_format(j.B, j.H, j.W, j.Cin, j.Cout, j.dgrad);
    PIS_CHECK_ARG(j.w && j.out && f != 0, "pis_conv3x3_filters: a job has no filter transform (no F(4x4,3x3) GEMM "
                                          "or direct path)");
    PIS_CHECK_ARG(j.out_bytes >= pis_conv3x3_filter_bytes(j.B, j.H, j.W, j.Cin, j.Cout, j.dgrad),
                  "pis_conv3x3_filters: a job's output is too small");
    if (f == 3) {
      dw[nd] = j.w; dout[nd] = j.out; dci[nd] = j.Cin; dco[nd] = j.Cout; ddg[nd] = j.dgrad ? 1 : 0;
      ++nd;
      continue;
    }
    w[nw] = j.w; out[nw] = j.out; fmt[nw] = f; dg[nw] = j.dgrad ? 1 : 0;
    C[nw] = j.dgrad ? j.Cout : j.Cin;  // contraction channels
    N[nw] = j.dgrad ? j.Cin : j.Cout;  // output channels
    ++nw;
  }
  int rc = nw ? launch_wino4_filter_batch(nw, w, out, C, N, dg, fmt, (hipStream_t)stream) : PIS_OK;
  if (!rc && nd) rc = launch_direct_wsplit_batch(nd, dw, dout, dci, dco, ddg, (hipStream_t)stream);
  return rc;
}

extern "C" int pis_conv3x3_dgrad(const float* dz, int ldz, const float* w_flip, const float* mask,
                                 int ldm, const float* scale, float* dx, int lddx, int B, int H,
                                 int W, int Cin, int Cout, int flags, pis_stream_t stream) {
  return pis_conv3x3_dgrad_ex(dz, ldz, w_flip, mask, ldm, scale, dx, lddx, B, H, W, Cin, Cout, flags, nullptr, 0,
                              stream);
}

extern "C" int pis_conv3x3_dgrad_ex(const float* dz, int ldz, const float* w_flip, const float* mask,
                                    int ldm, const float* scale, float* dx, int lddx, int B, int H,
                                    int W, int Cin, int Cout, int flags, void* ws, size_t ws_bytes,
                                    pis_stream_t stream) {
  PIS_CHECK_ARG(dz && w_flip && dx && B > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0,
                "pis_conv3x3_dgrad: bad arguments");
  PIS_CHECK_ARG(Cout % 4 == 0 && ldz % 4 == 0, "pis_conv3x3_dgrad: Cout/ldz must be multiples of 4");
  PIS_CHECK_ARG(!(flags & PIS_MASK) || mask, "pis_conv3x3_dgrad: PIS_MASK without mask");
  PIS_CHECK_ARG(!(flags & PIS_SCALE) || scale, "pis_conv3x3_dgrad: PIS_SCALE without scale");
  IGemmArgs a{};
  a.src = dz; a.lds = ldz; a.Hs = H; a.Ws = W; a.H = H; a.W = W; a.M = B * H * W;
  a.Csrc = Cout; a.ntaps = 9; a.tap_mode = TAP_CONV3; a.wt = w_flip; a.ldw = 9 * Cout; a.N = Cin;
  a.epi = EPI_NHWC; a.mask = mask; a.ldm = ldm; a.scale = scale; a.dst = dx; a.ldd = lddx;
  a.flags = flags & (PIS_MASK | PIS_SCALE | PIS_ACCUMULATE);
  a.w_unflipped = (flags & PIS_W_UNFLIPPED) != 0;
  a.filter_ready = (flags & PIS_FILTER_READY) != 0;
  a.is_dgrad = 1;
  PIS_CHECK_ARG(!a.w_unflipped || (flags & PIS_WINO_PREPARED) ||
                    (ws && direct_h3_wanted(H, W, Cout, Cin, ldz) && ws_bytes >= direct_h3_ws_bytes(Cout, Cin)) ||
                    (ws && wino6_layer(B, H, W, Cin, Cout) && wino_ok(a) && ws_bytes >= wino_ws_bytes(B, H, W, Cout, Cin)),
                "pis_conv3x3_dgrad_ex: PIS_W_UNFLIPPED needs the prepared F(4x4,3x3) path, the F(6x6,3x3) one or the "
                "direct one");
  return dispatch_conv3x3(a, B, ws, ws_bytes, (hipStream_t)stream, nullptr, (flags & PIS_WINO_PREPARED) != 0);
}

bool pis::dgrad_wino4_planned(int B, int H, int W, int Cin, int Cout, int ldz, size_t ws_bytes) {
  IGemmArgs a{};  // as pis_conv3x3_dgrad_ex builds it (dx / mask rows 16-B aligned)
  a.H = H; a.W = W; a.Csrc = Cout; a.N = Cin; a.lds = ldz; a.ldd = 4; a.ldm = 4;
  a.tap_mode = TAP_CONV3; a.epi = EPI_NHWC;
  return wino_ok(a) && wino_tile(H, W) == 4 && wino_wanted_dims(H, W, Cout, Cin) &&
         ws_bytes >= wino_ws_bytes(B, H, W, Cout, Cin) && !direct_h3_wanted(H, W, Cout, Cin, ldz) &&
         !wino6_layer(B, H, W, Cin, Cout);  // an F(6x6) input gradient transforms dz itself
}

// does pis_conv3x3_dgrad_ex take the direct fp16x3 kernel (which reads the original weights
// with PIS_W_UNFLIPPED, no flipped copy)?
extern "C" int pis_conv3x3_dgrad_direct(int B, int H, int W, int Cin, int Cout, int ldz, size_t ws_bytes) {
  return B > 0 && direct_h3_wanted(H, W, Cout, Cin, ldz) && ws_bytes >= direct_h3_ws_bytes(Cout, Cin);
}

extern "C" int pis_convt2x2_fwd(const float* x, int ldx, const float* w_ijoc, const float* bias,
                                float* y, int ldy, int B, int H, int W, int Cin, int Cout,
                                pis_stream_t stream) {
  PIS_CHECK_ARG(x && w_ijoc && y && B > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0,
                "pis_convt2x2_fwd: bad arguments");
  PIS_CHECK_ARG(Cin % 4 == 0 && ldx % 4 == 0, "pis_convt2x2_fwd: Cin/ldx must be multiples of 4");
  const int rc = launch_convt_gemm(0, x, ldx, w_ijoc, B, H, W, Cin, Cout, bias, nullptr, 0, y, ldy, 0,
                                   (hipStream_t)stream);
  if (rc <= 0) return rc;
  IGemmArgs a{};
  a.src = x; a.lds = ldx; a.Hs = H; a.Ws = W; a.H = H; a.W = W; a.M = B * H * W;
  a.Csrc = Cin; a.ntaps = 1; a.tap_mode = TAP_ONE; a.wt = w_ijoc; a.ldw = Cin; a.N = 4 * Cout;
  a.epi = EPI_SCATTER2; a.cout_t = Cout; a.bias = bias; a.dst = y; a.ldd = ldy; a.flags = 0;
  return launch_igemm(a, (hipStream_t)stream);
}

extern "C" int pis_convt2x2_prep(const float* w_ijoc, float* w_cijo, int Cin, int Cout,
                                 pis_stream_t stream) {
  PIS_CHECK_ARG(w_ijoc && w_cijo && Cin > 0 && Cout > 0, "pis_convt2x2_prep: bad arguments");
  const int64_t n = (int64_t)4 * Cin * Cout;
  const int grid = (int)std::min<int64_t>(cdiv(n, 256), 4096);
  hipLaunchKernelGGL(convt_prep_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, w_ijoc,
                     w_cijo, Cin, Cout);
  return launch_status("convt2x2_prep");
}

extern "C" int pis_convt2x2_dgrad(const float* dy, int lddy, const float* w_cijo, const float* mask,
                                  int ldm, float* dx, int lddx, int B, int H, int W, int Cin,
                                  int Cout, int flags, pis_stream_t stream) {
  PIS_CHECK_ARG(dy && w_cijo && dx && B > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0,
                "pis_convt2x2_dgrad: bad arguments");
  PIS_CHECK_ARG(Cout % 4 == 0 && lddy % 4 == 0, "pis_convt2x2_dgrad: Cout/lddy must be multiples of 4");
  PIS_CHECK_ARG(!(flags & PIS_MASK) || mask, "pis_convt2x2_dgrad: PIS_MASK without mask");
  const int rc = launch_convt_gemm(1, dy, lddy, w_cijo, B, H, W, Cin, Cout, nullptr, mask, ldm, dx, lddx,
                                   flags & (PIS_MASK | PIS_ACCUMULATE), (hipStream_t)stream);
  if (rc <= 0) return rc;
  IGemmArgs a{};
  a.src = dy; a.lds = lddy; a.Hs = 2 * H; a.Ws = 2 * W; a.H = H; a.W = W; a.M = B * H * W;
  a.Csrc = Cout; a.ntaps = 4; a.tap_mode = TAP_UP2; a.wt = w_cijo; a.ldw = 4 * Cout; a.N = Cin;
  a.epi = EPI_NHWC; a.mask = mask; a.ldm = ldm; a.dst = dx; a.ldd = lddx;
  a.flags = flags & (PIS_MASK | PIS_ACCUMULATE);
  return launch_igemm(a, (hipStream_t)stream);
}
