// Direct 3x3 convolution (padding 1) on the fp16 MFMA pipe in fp16x3 — src/unet.py:29,38's
// nn.Conv2d forward, and its input gradient (the same contraction over the flipped weights) —
// for the shallow U-Net layers, where the Winograd pipelines are bound by their transform
// traffic: no V / M / E intermediates, one read of the input tile (+ a 1-pixel
// halo) and one write of the output.
//
// Arithmetic (DESIGN §4 'fp16x3'): every operand is scaled by a power of two into fp16 range and
// split exactly into hi = fp16(v s), lo = fp16(v s - hi) (22 significant bits); each fp32
// product becomes lo*hi + hi*lo + hi*hi on v_mfma_f32_32x32x16_f16, accumulated in fp32.
// Scales: the weights one per output channel (max over taps and contraction channels into
// [2^13, 2^14)), written with the fp16 planes by conv3x3_wsplit_kernel; the input one per block
// and 16-channel chunk (its max over the staged halo tile, h3_keep), the accumulators re-expressed
// exactly when it changes; the epilogue divides once.
//
// Block = 256 threads (4 waves) = an 8 x 32 output-pixel tile x 64 output channels; wave w owns
// image rows 2w, 2w+1 of the tile (2 x 2 tiles of 32 pixels x 32 channels). Per 16-channel chunk:
// the 10 x 34 x 16 input halo (hi / lo planes, 21.8 KB) and the chunk's 9 x 64 x 16 weights
// (36.9 KB) are staged once in LDS, then 9 taps x 12 MFMAs per wave read shifted windows of the
// halo: the input is fetched 1.33x, its split amortised over 9 taps. Two blocks per CU (58.7 KB
// LDS each): one stages while the other computes. The next chunk's global loads are issued
// before this chunk's MFMAs and land meanwhile.
// LDS rows are 32 B (16 fp16); the two 16-B halves of row p are swapped when bit 3 of p is set:
// every ds_read_b128 lane group (16 lanes, any 16 consecutive rows, one half) and every
// ds_write_b128 group (8 lanes, 4 consecutive rows) then hits distinct bank slots.
#include "igemm.h"

namespace pis {

struct DirectArgs {
  const float* x;      // input NHWC (forward: x; input gradient: dz)
  int ldx;
  const _Float16* wp;  // conv3x3_wsplit_kernel's planes
  const float* winv;   // [N] 1 / t_n
  const float* bias;   // [N] or NULL
  const float* scale;  // [B][N] (PIS_SCALE)
  const float* mask;   // [B*H*W][ldm] (PIS_MASK: ReLU derivative of the conv's input)
  int ldm;
  float* y;
  int ldy;
  float* pool;         // [B][H/2][W/2][N] or NULL: also the 2x2 max pool of y
  int B, H, W, C, N;   // C contraction channels (% 16), N outputs (% 64)
  int flags;
};

constexpr int DT_H = 8, DT_W = 32, DH_H = DT_H + 2, DH_W = DT_W + 2, DH_P = DH_H * DH_W, DKC = 16;
constexpr int DX_BYTES = 2 * DH_P * DKC * 2;     // hi / lo halo planes
constexpr int DW_HALFS = 9 * 2 * 64 * DKC;       // one (chunk, 64-output slice) of the split weights
constexpr int DW_BYTES = DW_HALFS * 2;
constexpr int DX_ITEMS = 2 * DH_P;               // 8-channel halves of halo pixels
constexpr int DX_PER_T = (DX_ITEMS + 255) / 256; // 3
constexpr int DW_PER_T = DW_BYTES / 16 / 256;    // 9

__device__ __forceinline__ int dsw(int row, int half) { return row * DKC + 8 * (half ^ ((row >> 3) & 1)); }

// weights -> [chunk][slice][tap][plane][64][16] fp16 (rows swizzled as dsw), per output scale.
// dgrad = 0: out channel n, contraction c of w[n][r][s][c] (KRSC); dgrad = 1: out channel c,
// contraction n of the flipped filter w[n][2-r][2-s][c] (the input gradient).
__global__ __launch_bounds__(256) void conv3x3_wsplit_kernel(const float* __restrict__ w, int Cin, int Cout,
                                                             int dgrad, _Float16* __restrict__ out,
                                                             float* __restrict__ winv) {
  const int o = blockIdx.x;  // output channel of the contraction
  const int C = dgrad ? Cout : Cin, N = dgrad ? Cin : Cout, ns = N / 64;
  const int tid = threadIdx.x;
  auto at = [&](int tap, int k) -> float {
    const int r = tap / 3, s = tap % 3;
    return dgrad ? w[(((size_t)k * 3 + (2 - r)) * 3 + (2 - s)) * Cin + o] : w[((size_t)o * 9 + tap) * Cin + k];
  };
  float m = 0.f;
  for (int e = tid; e < 9 * C; e += 256) m = fmaxf(m, fabsf(at(e / C, e % C)));
  __shared__ float red[4];
  m = wave_max_nonneg(m);
  if ((tid & 63) == 0) red[tid >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  float t, inv;
  h2_scale_pair(m, t, inv);
  if (tid == 0) winv[o] = inv;
  const int slice = o / 64, row = o % 64;
  for (int e = tid; e < 9 * C; e += 256) {
    const int tap = e / C, k = e % C;
    const float v = at(tap, k) * t;
    const _Float16 hi = (_Float16)v, lo = (_Float16)(v - (float)hi);
    const size_t base = ((((size_t)(k / DKC) * ns + slice) * 9 + tap) * 2) * 64 * DKC;
    const int off = dsw(row, (k % DKC) >> 3) + (k & 7);
    out[base + off] = hi;
    out[base + 64 * DKC + off] = lo;
  }
}

template <bool POOL>
__global__ __launch_bounds__(256, 2) void conv3x3_h3_kernel(DirectArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[DX_BYTES + DW_BYTES + 64];
  _Float16* sx = reinterpret_cast<_Float16*>(smem);             // [plane][DH_P][16]
  _Float16* sw = reinterpret_cast<_Float16*>(smem + DX_BYTES);  // [tap][plane][64][16]
  float* red = reinterpret_cast<float*>(smem + DX_BYTES + DW_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 31, lh = lane >> 5;
  const int tw_n = g.W / DT_W, th_n = g.H / DT_H, per_img = tw_n * th_n, ntile = g.B * per_img;
  const int ns = g.N / 64;
  // the ns output slices of one pixel tile are dealt 8 apart (same XCD, back to back): the second
  // reads the input tile from L2
  const int bid = blockIdx.x;
  int gt, slice;
  if (ntile % 8 == 0) {
    gt = (bid / (8 * ns)) * 8 + bid % 8;
    slice = (bid / 8) % ns;
  } else {
    gt = bid / ns;
    slice = bid % ns;
  }
  const int b = gt / per_img, rem = gt - b * per_img, r0 = (rem / tw_n) * DT_H, c0 = (rem % tw_n) * DT_W;
  const int n0 = slice * 64;
  const float* xb = g.x + (size_t)b * g.H * g.W * g.ldx;
  const int nk = g.C / DKC;

  f32x4 xr[DX_PER_T][2];
  u32x4 wr[DW_PER_T];
  auto gload = [&](int k) {
#pragma unroll
    for (int j = 0; j < DX_PER_T; ++j) {
      const int i = tid + 256 * j;
      xr[j][0] = xr[j][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (i < DX_ITEMS) {
        const int q = i >> 1, h = i & 1, qr = q / DH_W, qc = q - qr * DH_W;
        const int row = r0 - 1 + qr, col = c0 - 1 + qc;
        if (row >= 0 && row < g.H && col >= 0 && col < g.W) {
          const float* p = xb + ((size_t)row * g.W + col) * g.ldx + k * DKC + 8 * h;
          xr[j][0] = *reinterpret_cast<const f32x4*>(p);
          xr[j][1] = *reinterpret_cast<const f32x4*>(p + 4);
        }
      }
    }
    const u32x4* wsrc = reinterpret_cast<const u32x4*>(g.wp + ((size_t)k * ns + slice) * DW_HALFS);
#pragma unroll
    for (int j = 0; j < DW_PER_T; ++j) wr[j] = wsrc[tid + 256 * j];
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  float s_cur = 0.f, s_min = __builtin_inff();

  gload(0);
#pragma unroll 1
  for (int k = 0; k < nk; ++k) {
    // 1. this chunk's weights into LDS; the halo's block-wide max
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < DX_PER_T; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) m = fmaxf(m, fmaxf(fabsf(xr[j][0][e]), fabsf(xr[j][1][e])));
    m = wave_max_nonneg(m);
    if (lane == 0) red[wave] = m;
#pragma unroll
    for (int j = 0; j < DW_PER_T; ++j) reinterpret_cast<u32x4*>(sw)[tid + 256 * j] = wr[j];
    __syncthreads();
    // 2. the chunk's scale (block-uniform); partial sums re-expressed in it; the split halo
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    const float s_new = h3_keep(s_cur, m, s_min);
    if (k > 0 && s_new != s_cur) {
      const float f = s_new / s_cur;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] *= f;
    }
    s_cur = s_new;
#pragma unroll
    for (int j = 0; j < DX_PER_T; ++j) {
      const int i = tid + 256 * j;
      if (i < DX_ITEMS) {
        const int q = i >> 1, h = i & 1;
        u32x2 h0, l0, h1, l1;
        split2h_x4(xr[j][0] * s_cur, h0, l0);
        split2h_x4(xr[j][1] * s_cur, h1, l1);
        *reinterpret_cast<u32x4*>(&sx[dsw(q, h)]) = u32x4{h0[0], h0[1], h1[0], h1[1]};
        *reinterpret_cast<u32x4*>(&sx[DH_P * DKC + dsw(q, h)]) = u32x4{l0[0], l0[1], l1[0], l1[1]};
      }
    }
    __syncthreads();
    // 3. the next chunk's loads fly during this chunk's MFMAs
    if (k + 1 < nk) gload(k + 1);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int r = tap / 3, s = tap % 3;
      f16x8 a[2][2], bb[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int p = (2 * wave + i + r) * DH_W + s + li;
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) a[i][pl] = *reinterpret_cast<const f16x8*>(&sx[pl * DH_P * DKC + dsw(p, lh)]);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
          bb[j][pl] = *reinterpret_cast<const f16x8*>(&sw[(tap * 2 + pl) * 64 * DKC + dsw(32 * j + li, lh)]);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {  // smallest partial products first
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i][1], bb[j][0], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i][0], bb[j][1], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[i][0], bb[j][0], acc[i][j], 0, 0, 0);
        }
    }
    __syncthreads();
  }

  // epilogue: lane (li, lh) holds, for output channel n0 + 32 j + li, image row r0 + 2 wave + i and
  // column c0 + (reg & 3) + 8 (reg >> 2) + 4 lh (the 32x32x16 C/D map)
  const float inv_s = 1.f / s_cur;  // exact: a power of two
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + 32 * j + li;
    const float wi = g.winv[n];
    const float bias = g.bias ? g.bias[n] : 0.f;
    const float sc = (g.flags & PIS_SCALE) ? g.scale[(size_t)b * g.N + n] : 1.f;
    float pm[2][8];  // POOL: this lane's column-pair maxima of row 2w + i
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int row = r0 + 2 * wave + i;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int col = c0 + (reg & 3) + 8 * (reg >> 2) + 4 * lh;
        const size_t pix = ((size_t)b * g.H + row) * g.W + col;
        float v = (acc[i][j][reg] * inv_s) * wi + bias;
        if (g.flags & PIS_RELU) v = fmaxf(v, 0.f);
        if ((g.flags & PIS_MASK) && !(g.mask[pix * g.ldm + n] > 0.f)) v = 0.f;
        v *= sc;
        float* dst = g.y + pix * g.ldy + n;
        if (g.flags & PIS_ACCUMULATE) v += *dst;
        *dst = v;
        if constexpr (POOL) {
          if (reg & 1) pm[i][reg >> 1] = fmaxf(pm[i][reg >> 1], v);
          else pm[i][reg >> 1] = v;
        }
      }
    }
    if constexpr (POOL) {
      const int prow = (r0 >> 1) + wave;
#pragma unroll
      for (int q = 0; q < 8; ++q) {  // column pair q: columns 2 (q & 1) + 8 (q >> 1) + 4 lh, +1
        const int pcol = (c0 >> 1) + (q & 1) + 4 * (q >> 1) + 2 * lh;
        g.pool[(((size_t)b * (g.H >> 1) + prow) * (g.W >> 1) + pcol) * g.N + n] = fmaxf(pm[0][q], pm[1][q]);
      }
    }
  }
}

bool direct_h3_shape_ok(int H, int W, int C, int N, int ldx) {
  return H % DT_H == 0 && W % DT_W == 0 && C % DKC == 0 && N % 64 == 0 && ldx % 4 == 0 && C >= DKC;
}

bool direct_h3_wanted(int H, int W, int C, int N, int ldx) {
  const int mode = tune_get(PIS_TUNE_DIRECT_H3);
  if (mode == 0 || !direct_h3_shape_ok(H, W, C, N, ldx)) return false;
  return mode == 2 || (C <= 128 && N <= 128 && H >= 256);
}

size_t direct_h3_ws_bytes(int C, int N) {
  return (size_t)9 * C * N * 2 * sizeof(_Float16) + (size_t)N * sizeof(float) + 256;
}

// a: the direct conv as pis_conv3x3_fwd_ex / _dgrad_ex build it (src = input, wt = KRSC weights,
// w_unflipped: an input gradient reading the ORIGINAL weights; otherwise a flipped copy w_flip
// [c][r][s][n], which is the forward layout of the transposed problem)
int launch_direct_h3(const IGemmArgs& a, int B, void* ws, size_t ws_bytes, hipStream_t s, bool dgrad_orig) {
  const int C = a.Csrc, N = a.N;
  if (!direct_h3_shape_ok(a.H, a.W, C, N, a.lds) || ws_bytes < direct_h3_ws_bytes(C, N))
    return set_error("direct conv: shape or workspace not supported"), PIS_ERR_ARG;
  _Float16* wp = reinterpret_cast<_Float16*>(ws);
  float* winv = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + (size_t)9 * C * N * 2 * sizeof(_Float16));
  // forward (or a flipped copy [Cin'=N][3][3][C] read as KRSC): out N, contraction C
  if (dgrad_orig)  // original weights w[C][3][3][N] (conv Cout = C, Cin = N): the flipped contraction
    hipLaunchKernelGGL(conv3x3_wsplit_kernel, dim3(N), dim3(256), 0, s, a.wt, N, C, 1, wp, winv);
  else
    hipLaunchKernelGGL(conv3x3_wsplit_kernel, dim3(N), dim3(256), 0, s, a.wt, C, N, 0, wp, winv);
  int rc = launch_status("conv3x3_wsplit");
  if (rc) return rc;
  DirectArgs g{};
  g.x = a.src; g.ldx = a.lds; g.wp = wp; g.winv = winv; g.bias = a.bias; g.scale = a.scale;
  g.mask = a.mask; g.ldm = a.ldm; g.y = a.dst; g.ldy = a.ldd; g.pool = a.pool;
  g.B = B; g.H = a.H; g.W = a.W; g.C = C; g.N = N; g.flags = a.flags;
  const int blocks = B * (a.H / DT_H) * (a.W / DT_W) * (N / 64);
  const double flop = 2.0 * 9 * (double)B * a.H * a.W * C * N;
  launch_hook("direct_h3", 0, s, flop);
  if (a.pool)
    hipLaunchKernelGGL(conv3x3_h3_kernel<true>, dim3(blocks), dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL(conv3x3_h3_kernel<false>, dim3(blocks), dim3(256), 0, s, g);
  launch_hook("direct_h3", 1, s, flop);
  return launch_status("conv3x3_h3");
}

}  // namespace pis
