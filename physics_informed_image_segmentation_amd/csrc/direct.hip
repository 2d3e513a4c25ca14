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
  int dbg;             // timing twins only (pis_tune key 2, wrong results; read only by the TW = true
                       // instantiations): 1 no global loads after the first chunk, 2 no LDS staging
                       // after the first chunk, 4 no epilogue
};

constexpr int DT_H = 8, DT_W = 32, DH_H = DT_H + 2, DH_W = DT_W + 2, DH_P = DH_H * DH_W, DKC = 16;
constexpr int DX_BYTES = 2 * DH_P * DKC * 2;     // hi / lo halo planes
constexpr int DW_HALFS = 9 * 2 * 64 * DKC;       // one (chunk, 64-output slice) of the split weights
constexpr int DW_BYTES = DW_HALFS * 2;
constexpr int DX_ITEMS = 2 * DH_P;               // 8-channel halves of halo pixels
constexpr int DX_PER_T = (DX_ITEMS + 255) / 256; // 3
constexpr int DW_PER_T = DW_BYTES / 16 / 256;    // 9

__device__ __forceinline__ f32x4 vmax4(f32x4 a, f32x4 b) {
  return f32x4{fmaxf(a[0], b[0]), fmaxf(a[1], b[1]), fmaxf(a[2], b[2]), fmaxf(a[3], b[3])};
}

__device__ __forceinline__ int dsw(int row, int half) { return row * DKC + 8 * (half ^ ((row >> 3) & 1)); }

// weights -> [chunk][slice][tap][plane][64][16] fp16 (rows swizzled as dsw), per output scale.
// dgrad = 0: out channel n, contraction c of w[n][r][s][c] (KRSC); dgrad = 1: out channel c,
// contraction n of the flipped filter w[n][2-r][2-s][c] (the input gradient).
struct WsplitJob {
  const float* w;  // KRSC [Cout][3][3][Cin]
  void* out;       // direct_h3_ws_bytes(C, N): the planes, then 1 / t_n
  int Cin, Cout, dgrad;
};
constexpr int WSPLIT_MAX_JOBS = 40;
struct WsplitBatch {
  WsplitJob j[WSPLIT_MAX_JOBS];
  int start[WSPLIT_MAX_JOBS + 1];
  int n;
};

__device__ __forceinline__ void wsplit_one(const float* __restrict__ w, int Cin, int Cout, int dgrad,
                                           _Float16* __restrict__ out, float* __restrict__ winv, int o) {
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

__global__ __launch_bounds__(256) void conv3x3_wsplit_kernel(const float* __restrict__ w, int Cin, int Cout,
                                                             int dgrad, _Float16* __restrict__ out,
                                                             float* __restrict__ winv) {
  wsplit_one(w, Cin, Cout, dgrad, out, winv, blockIdx.x);
}

// several layers' splits in ONE launch (pis_conv3x3_filters: PIS_FILTER_READY for the direct
// kernel): job k owns blocks [start[k], start[k + 1]), one per output channel of its contraction
__global__ __launch_bounds__(256) void conv3x3_wsplit_batch_kernel(WsplitBatch wb) {
  int k = 0;
  while (k + 1 < wb.n && (int)blockIdx.x >= wb.start[k + 1]) ++k;
  const WsplitJob& j = wb.j[k];
  const int C = j.dgrad ? j.Cout : j.Cin, N = j.dgrad ? j.Cin : j.Cout;
  _Float16* wp = reinterpret_cast<_Float16*>(j.out);
  float* winv = reinterpret_cast<float*>(reinterpret_cast<char*>(j.out) + (size_t)9 * C * N * 2 * sizeof(_Float16));
  wsplit_one(j.w, j.Cin, j.Cout, j.dgrad, wp, winv, (int)blockIdx.x - wb.start[k]);
}

// The direct kernels' epilogue (conv3x3_h3_kernel and the 8-wave form): the wave's rows r0 + 2 wave,
// + 1 from its accumulators, through its own 8 KB of LDS at E.
template <bool POOL, bool MPF, bool TW = false, int MPR = 2>  // MPR: mask rows prefetched (MPF); TW: timing twin
__device__ __forceinline__ void direct_epilogue(const DirectArgs& g, f32x16 (&acc)[2][2], float s_cur, float* E,
                                                const f32x4 (&mkp)[2][8], int b, int r0, int c0, int n0, int wave,
                                                int lane, int tid) {
  const int li = lane & 31, lh = lane >> 5, ch4 = 4 * (lane & 15);
  // epilogue: lane (li, lh) holds, for output channel n0 + 32 j + li, image row r0 + 2 wave + i and
  // column c0 + (reg & 3) + 8 (reg >> 2) + 4 lh (the 32x32x16 C/D map). Each image row goes through
  // the wave's own 8 KB of LDS ([32 px][64 ch], conflict-free both ways) so that every lane then
  // finishes 4 consecutive channels of 8 pixels with 16-B accesses: its mask / accumulate loads
  // are issued together (one memory round trip per row) and a pixel's 64 channels are one 256-B
  // store.
  const float inv_s = 1.f / s_cur;  // exact: a power of two
  if (TW && (g.dbg & 4)) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) t += acc[i][j][r];
    if (t == 1.2345f) g.y[tid] = t;
    return;
  }
  // float4 phase: lane (l & 15) owns channels n0 + ch4 .. + 3; pixel pair m = (l >> 4) + 4 k of the
  // row (columns 2m, 2m + 1: the 2x2 pool window's columns stay in one lane)
  const f32x4 wi4 = *reinterpret_cast<const f32x4*>(g.winv + n0 + ch4);
  const f32x4 bias4 = g.bias ? *reinterpret_cast<const f32x4*>(g.bias + n0 + ch4) : f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 sc4 = (g.flags & PIS_SCALE) ? *reinterpret_cast<const f32x4*>(g.scale + (size_t)b * g.N + n0 + ch4)
                                          : f32x4{1.f, 1.f, 1.f, 1.f};
  f32x4 prow0[4];  // POOL: row 2w's column-pair maxima
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = r0 + 2 * wave + i;
    const size_t pix0 = ((size_t)b * g.H + row) * g.W + c0;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) E[((reg & 3) + 8 * (reg >> 2) + 4 * lh) * 64 + 32 * j + li] = acc[i][j][reg];
    f32x4 mk[8], old[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const size_t pix = pix0 + 2 * ((lane >> 4) + 4 * (k >> 1)) + (k & 1);
      if (MPF && i < MPR && (g.flags & PIS_MASK))
        mk[k] = mkp[i][k];
      else
        mk[k] = (g.flags & PIS_MASK) ? *reinterpret_cast<const f32x4*>(g.mask + pix * g.ldm + n0 + ch4)
                                     : f32x4{1.f, 1.f, 1.f, 1.f};
      old[k] = (g.flags & PIS_ACCUMULATE) ? *reinterpret_cast<const f32x4*>(g.y + pix * g.ldy + n0 + ch4)
                                          : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int kp = 0; kp < 4; ++kp) {
      const int m = (lane >> 4) + 4 * kp;
      f32x4 v[2];
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const int k = 2 * kp + d;
        const f32x4 a = *reinterpret_cast<const f32x4*>(&E[(2 * m + d) * 64 + ch4]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float t = (a[e] * inv_s) * wi4[e] + bias4[e];
          if (g.flags & PIS_RELU) t = fmaxf(t, 0.f);
          if (!(mk[k][e] > 0.f)) t = 0.f;
          v[d][e] = t * sc4[e] + old[k][e];
        }
        *reinterpret_cast<f32x4*>(g.y + (pix0 + 2 * m + d) * g.ldy + n0 + ch4) = v[d];
      }
      if constexpr (POOL) {
        const f32x4 cm = vmax4(v[0], v[1]);
        if (i == 0) {
          prow0[kp] = cm;
        } else {
          const size_t pp = ((size_t)b * (g.H >> 1) + (r0 >> 1) + wave) * (g.W >> 1) + (c0 >> 1) + m;
          *reinterpret_cast<f32x4*>(g.pool + pp * g.N + n0 + ch4) = vmax4(prow0[kp], cm);
        }
      }
    }
  }
}

// MPF (pis_tune key 32 = 1, default): an input gradient's epilogue ReLU-mask rows are loaded
// during the last chunk's MFMAs (the last chunk is peeled), in the registers the absent next
// chunk's loads would use: enc1.conv1 input gradient -12 %, enc2.conv1 -4 % (profiles/r3_q18_*).
// (A tap loop walked column-shift-major, sharing halo rows between consecutive taps with the next
// tap's fragments issued ahead, measured neutral: the loop runs at the clock-limited MFMA rate.)
// TW: the timing-twin instantiation (pis_tune key 2 != 0 only); the production kernels carry no
// debug branch. DG: an input gradient — the same code, its own symbol, so that rocprofv3 and the PMC
// passes report forward, pooled forward and input gradient separately (the bench's per-role
// rooflines)
template <bool POOL, bool MPF = false, bool TW = false, bool DG = false>
__global__ __launch_bounds__(256, 2) void conv3x3_h3_kernel(DirectArgs g) {
  __shared__ __attribute__((aligned(16))) char smem[DX_BYTES + DW_BYTES + 64];
  _Float16* sx = reinterpret_cast<_Float16*>(smem);             // [plane][DH_P][16]
  _Float16* sw = reinterpret_cast<_Float16*>(smem + DX_BYTES);  // [tap][plane][64][16]
  float* red = reinterpret_cast<float*>(smem + DX_BYTES + DW_BYTES);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 31, lh = lane >> 5;
  const int tw_n = g.W / DT_W, th_n = g.H / DT_H, per_img = tw_n * th_n, ntile = g.B * per_img;
  const int ns = g.N / 64;
  const int nk = g.C / DKC;
  // block = (pixel tile, 64-output slice); the ns slices of one tile are dealt 8 apart (same XCD,
  // back to back: the second reads the input tile from L2). (A persistent grid walking the items,
  // prefetching the next item's first chunk during this one's MFMAs, measured 0.5-5 % slower per
  // layer and on the step: profiles/r3_q7_direct_grid.txt — co-resident blocks already hide it.)
  int gt, slice;
  if (ntile % 8 == 0) {
    gt = (blockIdx.x / (8 * ns)) * 8 + blockIdx.x % 8;
    slice = (blockIdx.x / 8) % ns;
  } else {
    gt = blockIdx.x / ns;
    slice = blockIdx.x % ns;
  }
  const int b = gt / per_img, rem = gt - b * per_img, r0 = (rem / tw_n) * DT_H, c0 = (rem % tw_n) * DT_W;
  const int n0 = slice * 64;
  const float* xb = g.x + (size_t)b * g.H * g.W * g.ldx;

  f32x4 xr[DX_PER_T][2];
  u32x4 wr[DW_PER_T];
  auto gload = [&](int k) {
    if (TW && (g.dbg & 1) && k > 0) return;
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

  // epilogue lane map (below): channels n0 + ch4 .. + 3 of pixel pair (lane >> 4) + 4 (k >> 1), k & 1
  const int ch4 = 4 * (lane & 15);
  f32x4 mkp[2][8];  // MPF: the ReLU-mask rows of the epilogue, loaded during the last chunk
  auto mask_prefetch = [&]() {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const size_t pix0 = ((size_t)b * g.H + r0 + 2 * wave + i) * g.W + c0;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const size_t pix = pix0 + 2 * ((lane >> 4) + 4 * (k >> 1)) + (k & 1);
        mkp[i][k] = *reinterpret_cast<const f32x4*>(g.mask + pix * g.ldm + n0 + ch4);
      }
    }
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
  // one chunk; the last one (peeled, LAST) issues the epilogue's mask loads instead of a next chunk's
  auto chunk = [&](int k, auto last_c) __attribute__((always_inline)) {
    constexpr bool LAST = decltype(last_c)::value;
    if (!(TW && (g.dbg & 2) && k > 0)) {
    // 1. this chunk's weights into LDS; the halo's block-wide max
    float m = wave_max_nonneg(absmax_x4(xr));
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
    }
    // 3. the next chunk's loads fly during this chunk's MFMAs
    if constexpr (!LAST) gload(k + 1);
    else if (MPF && (g.flags & PIS_MASK)) mask_prefetch();
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
  };
#pragma unroll 1
  for (int k = 0; k < nk - 1; ++k) chunk(k, std::false_type{});
  chunk(nk - 1, std::true_type{});

  // epilogue: the wave's 8 KB of LDS, free since the loop's last barrier
  direct_epilogue<POOL, MPF, TW>(g, acc, s_cur, reinterpret_cast<float*>(smem) + wave * (32 * 64), mkp, b, r0, c0, n0,
                             wave, lane, tid);
}


bool direct_h3_shape_ok(int H, int W, int C, int N, int ldx) {
  return H % DT_H == 0 && W % DT_W == 0 && C % DKC == 0 && N % 64 == 0 && ldx % 4 == 0 && C >= DKC;
}

bool direct_h3_wanted(int H, int W, int C, int N, int ldx) {
  const int mode = tune_get(PIS_TUNE_DIRECT_H3);
  if (mode == 0 || !direct_h3_shape_ok(H, W, C, N, ldx)) return false;
  const int lo = std::min(C, N), hi = std::max(C, N);
  if (mode == 3)  // + dec2.conv0 (256 <-> 128 at 256^2) and enc3.conv0 (128 <-> 256 at 128^2)
    return (H >= 256 && hi <= 256) || (H >= 128 && hi <= 256 && lo <= 128);
  if (mode == 4)  // + every <= 256-channel layer at 128^2 (enc3, dec3.conv1)
    return H >= 128 && hi <= 256;
  if (mode == 5)  // + every layer at 128^2 and above
    return H >= 128;
  return mode == 2 || (hi <= 128 && H >= 256);
}

// the direct kernel's weight splits of several layers in one launch (KRSC weights; dgrad: the
// contraction over Cout of the ORIGINAL weights, as launch_direct_h3's dgrad_orig)
int launch_direct_wsplit_batch(int n, const float* const* w, void* const* out, const int* Cin, const int* Cout,
                               const int* dgrad, hipStream_t s) {
  if (n <= 0) return PIS_OK;
  if (n > WSPLIT_MAX_JOBS) return set_error("direct wsplit batch: too many jobs"), PIS_ERR_ARG;
  WsplitBatch wb{};
  wb.n = n;
  int total = 0;
  for (int k = 0; k < n; ++k) {
    wb.j[k] = WsplitJob{w[k], out[k], Cin[k], Cout[k], dgrad[k]};
    wb.start[k] = total;
    total += dgrad[k] ? Cin[k] : Cout[k];
  }
  wb.start[n] = total;
  hipLaunchKernelGGL(conv3x3_wsplit_batch_kernel, dim3(total), dim3(256), 0, s, wb);
  return launch_status("conv3x3_wsplit_batch");
}

size_t direct_h3_ws_bytes(int C, int N) {
  return (size_t)9 * C * N * 2 * sizeof(_Float16) + (size_t)N * sizeof(float) + 256;
}

// a: the direct conv as pis_conv3x3_fwd_ex / _dgrad_ex build it (src = input, wt = KRSC weights,
// w_unflipped: an input gradient reading the ORIGINAL weights; otherwise a flipped copy w_flip
// [c][r][s][n], which is the forward layout of the transposed problem)
int launch_direct_h3(const IGemmArgs& a, int B, void* ws, size_t ws_bytes, hipStream_t s, bool dgrad_orig,
                     bool ready) {
  const int C = a.Csrc, N = a.N;
  if (!direct_h3_shape_ok(a.H, a.W, C, N, a.lds) || (!ready && ws_bytes < direct_h3_ws_bytes(C, N)))
    return set_error("direct conv: shape or workspace not supported"), PIS_ERR_ARG;
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (!a16(a.src) || !a16(a.dst) || a.ldd % 4 || ((a.flags & PIS_MASK) && (!a16(a.mask) || a.ldm % 4)) ||
      (a.pool && !a16(a.pool)) || ((a.flags & PIS_SCALE) && !a16(a.scale)) || (a.bias && !a16(a.bias)))
    return set_error("direct conv: input, output, mask, scale, bias and pool must be 16-byte aligned with "
                     "channel strides % 4 == 0"), PIS_ERR_ARG;
  // ready (PIS_FILTER_READY): a.wt IS the split — planes, then 1 / t_n — from pis_conv3x3_filter(s)
  void* wsp = ready ? const_cast<float*>(a.wt) : ws;
  _Float16* wp = reinterpret_cast<_Float16*>(wsp);
  float* winv = reinterpret_cast<float*>(reinterpret_cast<char*>(wsp) + (size_t)9 * C * N * 2 * sizeof(_Float16));
  if (!ready) {
    // forward (or a flipped copy [Cin'=N][3][3][C] read as KRSC): out N, contraction C
    if (dgrad_orig)  // original weights w[C][3][3][N] (conv Cout = C, Cin = N): the flipped contraction
      hipLaunchKernelGGL(conv3x3_wsplit_kernel, dim3(N), dim3(256), 0, s, a.wt, N, C, 1, wp, winv);
    else
      hipLaunchKernelGGL(conv3x3_wsplit_kernel, dim3(N), dim3(256), 0, s, a.wt, C, N, 0, wp, winv);
    const int rc = launch_status("conv3x3_wsplit");
    if (rc) return rc;
  } else if (((uintptr_t)wsp & 15) != 0) {
    return set_error("direct conv: the ready split must be 16-byte aligned"), PIS_ERR_ARG;
  }
  DirectArgs g{};
  g.x = a.src; g.ldx = a.lds; g.wp = wp; g.winv = winv; g.bias = a.bias; g.scale = a.scale;
  g.mask = a.mask; g.ldm = a.ldm; g.y = a.dst; g.ldy = a.ldd; g.pool = a.pool;
  g.B = B; g.H = a.H; g.W = a.W; g.C = C; g.N = N; g.flags = a.flags;
  g.dbg = tune_get(PIS_TUNE_DEBUG_NOLOAD);
  const double flop = 2.0 * 9 * (double)B * a.H * a.W * C * N;
  const bool mpf = tune_get(PIS_TUNE_DIRECT_PIPE) != 0 && (a.flags & PIS_MASK);
  const int blocks = B * (a.H / DT_H) * (a.W / DT_W) * (N / 64);
  // the launch hook's label names the role: pooled forward, forward, input gradient
  const char* role = a.pool ? "direct_h3_pool" : a.is_dgrad ? "direct_h3_dgrad" : "direct_h3_fwd";
  const dim3 grid(blocks);
  launch_hook(role, 0, s, flop);
  if (g.dbg) {  // timing twins (tools/bench_kernels.py --dbg): wrong results by design
    if (a.pool)
      hipLaunchKernelGGL((conv3x3_h3_kernel<true, false, true>), grid, dim3(256), 0, s, g);
    else if (mpf)
      hipLaunchKernelGGL((conv3x3_h3_kernel<false, true, true>), grid, dim3(256), 0, s, g);
    else
      hipLaunchKernelGGL((conv3x3_h3_kernel<false, false, true>), grid, dim3(256), 0, s, g);
  } else if (a.pool) {  // a forward: no mask
    hipLaunchKernelGGL((conv3x3_h3_kernel<true, false>), grid, dim3(256), 0, s, g);
  } else if (!a.is_dgrad) {
    hipLaunchKernelGGL((conv3x3_h3_kernel<false, false>), grid, dim3(256), 0, s, g);
  } else if (mpf) {
    hipLaunchKernelGGL((conv3x3_h3_kernel<false, true, false, true>), grid, dim3(256), 0, s, g);
  } else {
    hipLaunchKernelGGL((conv3x3_h3_kernel<false, false, false, true>), grid, dim3(256), 0, s, g);
  }
  launch_hook(role, 1, s, flop);
  return launch_status("conv3x3_h3");
}


// =============================================================================================
// Weight gradient of the direct conv (src/unet.py:29,38's backward w.r.t. the conv's weight and
// bias): dW[n][r][s][c] = sum_p dz[p][n] x[p + (r-1, s-1)][c], db[n] = sum_p dz[p][n], in fp16x3.
// GEMM view: rows n (64 per block), columns (tap, c) (9 x 64 per block), contraction over pixels.
// A block walks pixel tiles of 4 rows x 32 columns (split-K: tiles split, split + splits, ...):
// per tile the dz tile (128 px x 64 n) and the x halo (6 x 34 px x 64 c), each in hi / lo fp16
// planes with one power-of-two scale per tile and operand (block-wide max, h3_keep), are staged
// in LDS as [pixel][channel] rows, and the MFMA operands — k = 8 consecutive pixels of one channel
// per lane — come out of them by transposed reads (ds_read_b64_tr_b16: 4 pixels x 16 channels per
// 16-lane group), the tap shift being a per-lane row address. Wave w: n-half w >> 1, c-half w & 1,
// all 9 taps (9 accumulator tiles of 32 x 32). One block per CU (85 KB LDS, ~290 registers per
// lane), the next tile's global loads in flight during this tile's 216 MFMAs per wave. Partial
// sums per block go to fp32 slabs [split][Cout][9][Cin] (reduce_slabs: fixed order, deterministic)
// and the bias partials to [split][Cout].
// LDS rows are 128 B (64 fp16); the 16-B chunk index is XORed with bit 1 of the row, shifted to
// bit 2: a transposed read's 32-lane half (4 consecutive rows x 64 B) then hits 64 distinct banks.
// =============================================================================================

struct DirectWArgs {
  const float* x;
  int ldx;
  const float* dz;
  int ldz;
  float* part;       // [splits][Cout][9][Cin]
  float* part_bias;  // [splits][Cout] or NULL
  int B, H, W, Cin, Cout, splits;
  int dbg;           // timing twins, as DirectArgs::dbg
  int vwalk;         // 4-row kernel (pis_tune key 43): 1 contiguous tile runs walked down the columns
};

constexpr int WT_H = 4, WT_W = 32, WT_P = WT_H * WT_W, WH_H = WT_H + 2, WH_W = WT_W + 2, WH_P = WH_H * WH_W;
constexpr int WZ_HALFS = WT_P * 64, WX_HALFS = WH_P * 64;                 // per plane
constexpr int WZ_ITEMS = WT_P * 8, WX_ITEMS = WH_P * 8;                   // 8-channel groups
constexpr int WLDS_BYTES = 2 * (WZ_HALFS + WX_HALFS) * 2;

// element offset of channel group (16-B chunk) ch of row `row` in a [row][64] fp16 image
__device__ __forceinline__ int wsw64(int row, int ch) { return row * 64 + 8 * (ch ^ (((row >> 1) & 1) << 2)); }

// (An eight-wave form — the taps split between the wave halves, 80 accumulator registers, two
// waves per SIMD — measured within +-2 % per layer, profiles/r3_q19_wg8.txt: not kept.)
template <bool TW = false>  // TW: timing twin (pis_tune key 2 != 0 only)
__global__ __launch_bounds__(256, 1) void conv3x3_wgrad_h3_kernel(DirectWArgs g) {
  constexpr int NW = 4, NT = 64 * NW, WZ_PER_T = WZ_ITEMS / NT, WX_PER_T = (WX_ITEMS + NT - 1) / NT;
  constexpr int NTAP = 9;
  __shared__ __attribute__((aligned(16))) char smem[WLDS_BYTES + 64];
  _Float16* sz = reinterpret_cast<_Float16*>(smem);                        // [plane][128][64]
  _Float16* sx = reinterpret_cast<_Float16*>(smem + 2 * WZ_HALFS * 2);     // [plane][204][64]
  float* red = reinterpret_cast<float*>(smem + WLDS_BYTES);                // [2][NW] wave maxima
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = (wave >> 1) & 1, wj = wave & 1;  // n-half, c-half
  constexpr int tap0 = 0, ntap = 9;
  const int ncb = g.Cin / 64, pairs = (g.Cout / 64) * ncb;
  // vwalk (key 43): a block owns a contiguous run of tiles ordered row-quad fastest, so consecutive
  // tiles are vertical neighbours sharing two x halo rows (fetched a tile ago: L2 hits, x read from
  // HBM ~1.06x instead of 1.59x), and the pairs of one split go to one XCD back to back (they share
  // its dz / x tiles); else tiles t = split, split + splits, ... in row-major order
  int pair, split;
  if (g.vwalk && (g.splits & 7) == 0) {
    const int bid = blockIdx.x, xcd = bid & 7, j = bid >> 3;
    pair = j % pairs;
    split = (j / pairs) * 8 + xcd;
  } else {
    pair = blockIdx.x % pairs;
    split = blockIdx.x / pairs;
  }
  const int n0 = (pair / ncb) * 64, c0 = (pair % ncb) * 64;
  const int tw_n = g.W / WT_W, nrq = g.H / WT_H, per_img = nrq * tw_n, ntile = g.B * per_img;
  const bool do_bias = g.part_bias != nullptr && c0 == 0;
  const int tps = (ntile + g.splits - 1) / g.splits;
  const int t_begin = g.vwalk ? split * tps : split, t_end = g.vwalk ? min(ntile, t_begin + tps) : ntile;
  const int t_step = g.vwalk ? 1 : g.splits;

  f32x4 zr[WZ_PER_T][2], xr[WX_PER_T][2];
  auto gload = [&](int t) {
    if (TW && (g.dbg & 1) && t != t_begin) return;
    const int b = t / per_img, rem = t - b * per_img;
    const int pr0 = (g.vwalk ? rem % nrq : rem / tw_n) * WT_H, pc0 = (g.vwalk ? rem / nrq : rem % tw_n) * WT_W;
    const size_t img = (size_t)b * g.H * g.W;
#pragma unroll
    for (int j = 0; j < WZ_PER_T; ++j) {
      const int i = tid + NT * j, px = i >> 3, cg = i & 7;
      const float* p = g.dz + (img + (size_t)(pr0 + (px >> 5)) * g.W + pc0 + (px & 31)) * g.ldz + n0 + 8 * cg;
      zr[j][0] = *reinterpret_cast<const f32x4*>(p);
      zr[j][1] = *reinterpret_cast<const f32x4*>(p + 4);
    }
#pragma unroll
    for (int j = 0; j < WX_PER_T; ++j) {
      const int i = tid + NT * j, q = i >> 3, cg = i & 7;
      xr[j][0] = xr[j][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (i < WX_ITEMS) {
        const int qr = q / WH_W, qc = q - qr * WH_W, row = pr0 - 1 + qr, col = pc0 - 1 + qc;
        if (row >= 0 && row < g.H && col >= 0 && col < g.W) {
          const float* p = g.x + (img + (size_t)row * g.W + col) * g.ldx + c0 + 8 * cg;
          xr[j][0] = *reinterpret_cast<const f32x4*>(p);
          xr[j][1] = *reinterpret_cast<const f32x4*>(p + 4);
        }
      }
    }
  };

  f32x16 acc[NTAP];
#pragma unroll
  for (int t = 0; t < NTAP; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // bias partials: channels n0 + 8 (tid & 7) + e
  float sz_cur = 0.f, sx_cur = 0.f, sz_min = __builtin_inff(), sx_min = __builtin_inff();

  // lane roles in the transposed reads: 16-lane group gq, its row q and 8-B column slot p
  const int gq = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int kh = gq >> 1;  // k half (pixels 8 kh ..)
  const int cgA = 4 * wi + 2 * (gq & 1) + (p >> 1), cgB = 4 * wj + 2 * (gq & 1) + (p >> 1);

  int t = t_begin;
  if (t < t_end) gload(t);
#pragma unroll 1
  for (; t < t_end; t += t_step) {
    if (!(TW && (g.dbg & 2) && t != t_begin)) {
    // 1. block maxima of the staged operands
    float mz = wave_max_nonneg(absmax_x4(zr));
    float mx = wave_max_nonneg(absmax_x4(xr));
    if (lane == 0) {
      red[wave] = mz;
      red[NW + wave] = mx;
    }
    if (do_bias) {
#pragma unroll
      for (int j = 0; j < WZ_PER_T; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bs[e] += zr[j][0][e];
          bs[4 + e] += zr[j][1][e];
        }
    }
    __syncthreads();
    // 2. this tile's scales; the partial sums re-expressed in them; split into LDS
    mz = red[0];
    mx = red[NW];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      mz = fmaxf(mz, red[w]);
      mx = fmaxf(mx, red[NW + w]);
    }
    const float sz_new = h3_keep(sz_cur, mz, sz_min), sx_new = h3_keep(sx_cur, mx, sx_min);
    if (sz_cur > 0.f && (sz_new != sz_cur || sx_new != sx_cur)) {
      const float f = (sz_new / sz_cur) * (sx_new / sx_cur);
#pragma unroll
      for (int k = 0; k < NTAP; ++k) acc[k] *= f;
    }
    sz_cur = sz_new;
    sx_cur = sx_new;
#pragma unroll
    for (int j = 0; j < WZ_PER_T; ++j) {
      const int i = tid + NT * j, px = i >> 3, cg = i & 7;
      u32x2 h0, l0, h1, l1;
      split2h_x4(zr[j][0] * sz_cur, h0, l0);
      split2h_x4(zr[j][1] * sz_cur, h1, l1);
      *reinterpret_cast<u32x4*>(&sz[wsw64(px, cg)]) = u32x4{h0[0], h0[1], h1[0], h1[1]};
      *reinterpret_cast<u32x4*>(&sz[WZ_HALFS + wsw64(px, cg)]) = u32x4{l0[0], l0[1], l1[0], l1[1]};
    }
#pragma unroll
    for (int j = 0; j < WX_PER_T; ++j) {
      const int i = tid + NT * j, qq = i >> 3, cg = i & 7;
      if (i < WX_ITEMS) {
        u32x2 h0, l0, h1, l1;
        split2h_x4(xr[j][0] * sx_cur, h0, l0);
        split2h_x4(xr[j][1] * sx_cur, h1, l1);
        *reinterpret_cast<u32x4*>(&sx[wsw64(qq, cg)]) = u32x4{h0[0], h0[1], h1[0], h1[1]};
        *reinterpret_cast<u32x4*>(&sx[WX_HALFS + wsw64(qq, cg)]) = u32x4{l0[0], l0[1], l1[0], l1[1]};
      }
    }
    __syncthreads();
    }
    // 3. the next tile's loads fly during this tile's MFMAs
    if (t + t_step < t_end) gload(t + t_step);
    // Halo-row-major: the 8 A fragments (tile row rr, column half cc: pixels 16 (2 rr + cc) + 8 kh +
    // q (+ 4), channels of cgA) are read once; then for each halo row h and column half cc the 3 B
    // fragments (halo pixel (h, 16 cc + 8 kh + q (+ 4) + s), channels of cgB) serve every tap row r
    // with rr = h - r. Each accumulator still takes its (rr, cc) contributions in K-step order
    // 2 rr + cc, three MFMAs each in the same order, so the sums are bitwise those of a loop over
    // 16-pixel K-steps — but each B fragment is read once per tile, one step AHEAD: the
    // sched_group_barriers issue step st + 1's 12 reads before step st's 9-27 MFMAs, whose time
    // hides their latency (the compiler's own schedule waited on each tap's reads right before its
    // MFMAs: lgkmcnt(0) inside the MFMA stream, profiles/r4_w_*).
    f16x8 af[4][2][2];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
#pragma unroll
      for (int cc = 0; cc < 2; ++cc)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) {
          const _Float16* base = sz + pl * WZ_HALFS;
          const int px = 16 * (2 * rr + cc) + 8 * kh + q;
          const s16x4 lo4 = tr_read(base + wsw64(px, cgA) + 4 * (p & 1));
          const s16x4 hi4 = tr_read(base + wsw64(px + 4, cgA) + 4 * (p & 1));
          af[rr][cc][pl] = __builtin_bit_cast(f16x8, __builtin_shufflevector(lo4, hi4, 0, 1, 2, 3, 4, 5, 6, 7));
        }
    f16x8 bf[2][3][2];
    auto bload = [&](int st, int buf) __attribute__((always_inline)) {
      const int h = st >> 1, cc0 = 16 * (st & 1);
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int hp = h * WH_W + cc0 + 8 * kh + q + s;
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) {
          const _Float16* base = sx + pl * WX_HALFS;
          const s16x4 lo4 = tr_read(base + wsw64(hp, cgB) + 4 * (p & 1));
          const s16x4 hi4 = tr_read(base + wsw64(hp + 4, cgB) + 4 * (p & 1));
          bf[buf][s][pl] = __builtin_bit_cast(f16x8, __builtin_shufflevector(lo4, hi4, 0, 1, 2, 3, 4, 5, 6, 7));
        }
      }
    };
    bload(0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 44, 0);  // LDS reads: the A fragments, step 0's B
#pragma unroll
    for (int st = 0; st < 12; ++st) {  // (h, cc) = (st >> 1, st & 1)
      const int h = st >> 1, cc = st & 1, cur = st & 1;
      if (st + 1 < 12) bload(st + 1, cur ^ 1);
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int rr = h - r;
        if (rr < 0 || rr > 3) continue;
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int tt = 3 * r + s;
          acc[tt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[rr][cc][1], bf[cur][s][0], acc[tt], 0, 0, 0);
          acc[tt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[rr][cc][0], bf[cur][s][1], acc[tt], 0, 0, 0);
          acc[tt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[rr][cc][0], bf[cur][s][0], acc[tt], 0, 0, 0);
        }
      }
      if (st + 1 < 12) __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);  // next step's reads,
      if (h == 0 || h == 5)                                                  // then this step's MFMAs
        __builtin_amdgcn_sched_group_barrier(0x008, 9, 0);
      else if (h == 1 || h == 4)
        __builtin_amdgcn_sched_group_barrier(0x008, 18, 0);
      else
        __builtin_amdgcn_sched_group_barrier(0x008, 27, 0);
    }
    __syncthreads();
  }

  // partial sums / (sz sx) -> slab [split][Cout][9][Cin]: lane column c0 + 32 wj + (lane & 31),
  // rows n0 + 32 wi + (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
  const float inv = (sz_cur > 0.f) ? (1.f / sz_cur) * (1.f / sx_cur) : 0.f;
  float* slab = g.part + (size_t)split * g.Cout * 9 * g.Cin;
  const int c = c0 + 32 * wj + (lane & 31);
#pragma unroll
  for (int tt = 0; tt < ntap; ++tt) {
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int n = n0 + 32 * wi + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
      slab[((size_t)n * 9 + tap0 + tt) * g.Cin + c] = acc[tt][reg] * inv;
    }
  }
  if (do_bias) {  // fixed-order reduction over the 32 threads of each channel group
    float* rb = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int e = 0; e < 8; ++e) rb[tid * 8 + e] = bs[e];
    __syncthreads();
    if (tid < 64) {
      const int cg = tid >> 3, e = tid & 7;
      float sum = 0.f;
      for (int k = 0; k < NT / 8; ++k) sum += rb[(8 * k + cg) * 8 + e];
      g.part_bias[(size_t)split * g.Cout + n0 + tid] = sum;
    }
  }
}


// The same weight gradient on TH-row tiles (pis_tune key 49 = TH = 2): two blocks per CU instead of
// one. The 4-row kernel above runs ONE wave per SIMD (85 KB LDS, ~290 registers), so nothing hides
// its staging (global loads, block maxima, split, LDS stores: ~35 % of its time, the timing twins
// of profiles/r4_h_*). Here a tile is TH x 32 pixels: dz 64 px x 64 ch and the (TH + 2) x 34 x halo
// in hi / lo planes = 51 KB of LDS at TH = 2, no register prefetch of the next tile (its loads are
// issued at the top of each tile: the second block of the CU computes meanwhile), <= 256 registers
// -> two independent blocks per CU, one staging while the other multiplies. Same per-tile
// arithmetic as the 4-row kernel (tile scales, halo-row-major MFMA order); the sums differ from it
// only by the tile grouping (fp32-class either way; tests/test_direct_gpu.py).
template <int TH>
__global__ __launch_bounds__(256, 2) void conv3x3_wgrad_h3r_kernel(DirectWArgs g) {
  constexpr int NW = 4, NT = 64 * NW, NTAP = 9;
  constexpr int TP = TH * WT_W, HHh = TH + 2, HP = HHh * WH_W;  // tile pixels, halo rows, halo pixels
  constexpr int ZH = TP * 64, XH = HP * 64;                       // fp16 per plane
  constexpr int ZI = TP * 8, XI = HP * 8;                         // 8-channel groups
  constexpr int Z_PER_T = ZI / NT, X_PER_T = (XI + NT - 1) / NT;
  static_assert(ZI % NT == 0, "dz items tile the block");
  __shared__ __attribute__((aligned(16))) char smem[2 * (ZH + XH) * 2 + 64];
  _Float16* sz = reinterpret_cast<_Float16*>(smem);
  _Float16* sx = reinterpret_cast<_Float16*>(smem + 2 * ZH * 2);
  float* red = reinterpret_cast<float*>(smem + 2 * (ZH + XH) * 2);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = (wave >> 1) & 1, wj = wave & 1;  // n-half, c-half
  const int ncb = g.Cin / 64, pairs = (g.Cout / 64) * ncb;
  int pair, split;
  if (g.vwalk && (g.splits & 7) == 0) {
    const int bid = blockIdx.x, xcd = bid & 7, j = bid >> 3;
    pair = j % pairs;
    split = (j / pairs) * 8 + xcd;
  } else {
    pair = blockIdx.x % pairs;
    split = blockIdx.x / pairs;
  }
  const int n0 = (pair / ncb) * 64, c0 = (pair % ncb) * 64;
  const int tw_n = g.W / WT_W, nrq = g.H / TH, per_img = nrq * tw_n, ntile = g.B * per_img;
  const bool do_bias = g.part_bias != nullptr && c0 == 0;
  const int tps = (ntile + g.splits - 1) / g.splits;
  const int t_begin = g.vwalk ? split * tps : split, t_end = g.vwalk ? min(ntile, t_begin + tps) : ntile;
  const int t_step = g.vwalk ? 1 : g.splits;

  f32x16 acc[NTAP];
#pragma unroll
  for (int t = 0; t < NTAP; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float sz_cur = 0.f, sx_cur = 0.f, sz_min = __builtin_inff(), sx_min = __builtin_inff();
  const int gq = lane >> 4, q0 = (lane & 15) >> 2, p = lane & 3;
  const int kh0 = gq >> 1;
  const int cgA0 = 4 * wi + 2 * (gq & 1) + (p >> 1), cgB0 = 4 * wj + 2 * (gq & 1) + (p >> 1);

#pragma unroll 1
  for (int t = t_begin; t < t_end; t += t_step) {
    // 1. this tile's global loads, block maxima
    f32x4 zr[Z_PER_T][2], xr[X_PER_T][2];
    {
      const int b = t / per_img, rem = t - b * per_img;
      const int pr0 = (g.vwalk ? rem % nrq : rem / tw_n) * TH, pc0 = (g.vwalk ? rem / nrq : rem % tw_n) * WT_W;
      const size_t img = (size_t)b * g.H * g.W;
#pragma unroll
      for (int j = 0; j < Z_PER_T; ++j) {
        const int i = tid + NT * j, px = i >> 3, cg = i & 7;
        const float* pz = g.dz + (img + (size_t)(pr0 + (px >> 5)) * g.W + pc0 + (px & 31)) * g.ldz + n0 + 8 * cg;
        zr[j][0] = *reinterpret_cast<const f32x4*>(pz);
        zr[j][1] = *reinterpret_cast<const f32x4*>(pz + 4);
      }
#pragma unroll
      for (int j = 0; j < X_PER_T; ++j) {
        const int i = tid + NT * j, qq = i >> 3, cg = i & 7;
        xr[j][0] = xr[j][1] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (i < XI) {
          const int qr = qq / WH_W, qc = qq - qr * WH_W, row = pr0 - 1 + qr, col = pc0 - 1 + qc;
          if (row >= 0 && row < g.H && col >= 0 && col < g.W) {
            const float* px_ = g.x + (img + (size_t)row * g.W + col) * g.ldx + c0 + 8 * cg;
            xr[j][0] = *reinterpret_cast<const f32x4*>(px_);
            xr[j][1] = *reinterpret_cast<const f32x4*>(px_ + 4);
          }
        }
      }
    }
    float mz = wave_max_nonneg(absmax_x4(zr));
    float mx = wave_max_nonneg(absmax_x4(xr));
    if (lane == 0) {
      red[wave] = mz;
      red[NW + wave] = mx;
    }
    if (do_bias) {
#pragma unroll
      for (int j = 0; j < Z_PER_T; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bs[e] += zr[j][0][e];
          bs[4 + e] += zr[j][1][e];
        }
    }
    __syncthreads();  // also: the previous tile's fragment reads are done
    // 2. scales, accumulators re-expressed, split into LDS
    mz = red[0];
    mx = red[NW];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      mz = fmaxf(mz, red[w]);
      mx = fmaxf(mx, red[NW + w]);
    }
    const float sz_new = h3_keep(sz_cur, mz, sz_min), sx_new = h3_keep(sx_cur, mx, sx_min);
    if (sz_cur > 0.f && (sz_new != sz_cur || sx_new != sx_cur)) {
      const float f = (sz_new / sz_cur) * (sx_new / sx_cur);
#pragma unroll
      for (int k = 0; k < NTAP; ++k) acc[k] *= f;
    }
    sz_cur = sz_new;
    sx_cur = sx_new;
#pragma unroll
    for (int j = 0; j < Z_PER_T; ++j) {
      const int i = tid + NT * j, px = i >> 3, cg = i & 7;
      u32x2 h0, l0, h1, l1;
      split2h_x4(zr[j][0] * sz_cur, h0, l0);
      split2h_x4(zr[j][1] * sz_cur, h1, l1);
      *reinterpret_cast<u32x4*>(&sz[wsw64(px, cg)]) = u32x4{h0[0], h0[1], h1[0], h1[1]};
      *reinterpret_cast<u32x4*>(&sz[ZH + wsw64(px, cg)]) = u32x4{l0[0], l0[1], l1[0], l1[1]};
    }
#pragma unroll
    for (int j = 0; j < X_PER_T; ++j) {
      const int i = tid + NT * j, qq = i >> 3, cg = i & 7;
      if (i < XI) {
        u32x2 h0, l0, h1, l1;
        split2h_x4(xr[j][0] * sx_cur, h0, l0);
        split2h_x4(xr[j][1] * sx_cur, h1, l1);
        *reinterpret_cast<u32x4*>(&sx[wsw64(qq, cg)]) = u32x4{h0[0], h0[1], h1[0], h1[1]};
        *reinterpret_cast<u32x4*>(&sx[XH + wsw64(qq, cg)]) = u32x4{l0[0], l0[1], l1[0], l1[1]};
      }
    }
    __syncthreads();
    // 3. halo-row-major MFMA phase (as the 4-row kernel): A fragments once per tile, each B fragment
    // once per halo row
    // the fragment addresses are tile-invariant: laundered per tile so the compiler recomputes them
    // instead of keeping ~100 of them live across the tile loop (two waves per SIMD: <= 256 registers)
    int q = q0, kh = kh0, cgA = cgA0, cgB = cgB0;
    asm volatile("" : "+v"(q), "+v"(kh), "+v"(cgA), "+v"(cgB));
    f16x8 af[TH][2][2];
#pragma unroll
    for (int rr = 0; rr < TH; ++rr)
#pragma unroll
      for (int cc = 0; cc < 2; ++cc)
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) {
          const _Float16* base = sz + pl * ZH;
          const int px = 16 * (2 * rr + cc) + 8 * kh + q;
          const s16x4 lo4 = tr_read(base + wsw64(px, cgA) + 4 * (p & 1));
          const s16x4 hi4 = tr_read(base + wsw64(px + 4, cgA) + 4 * (p & 1));
          af[rr][cc][pl] = __builtin_bit_cast(f16x8, __builtin_shufflevector(lo4, hi4, 0, 1, 2, 3, 4, 5, 6, 7));
        }
    // one B fragment set (registers: two waves per SIMD need <= 256; the SIMD's other wave hides
    // the LDS latency the 4-row kernel's read-ahead set hides)
    f16x8 bf[3][2];
#pragma unroll
    for (int st = 0; st < 2 * HHh; ++st) {  // (h, cc) = (st >> 1, st & 1)
      const int h = st >> 1, cc = st & 1;
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int hp = h * WH_W + 16 * cc + 8 * kh + q + s;
#pragma unroll
        for (int pl = 0; pl < 2; ++pl) {
          const _Float16* base = sx + pl * XH;
          const s16x4 lo4 = tr_read(base + wsw64(hp, cgB) + 4 * (p & 1));
          const s16x4 hi4 = tr_read(base + wsw64(hp + 4, cgB) + 4 * (p & 1));
          bf[s][pl] = __builtin_bit_cast(f16x8, __builtin_shufflevector(lo4, hi4, 0, 1, 2, 3, 4, 5, 6, 7));
        }
      }
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int rr = h - r;
        if (rr < 0 || rr >= TH) continue;
#pragma unroll
        for (int s = 0; s < 3; ++s) {
          const int tt = 3 * r + s;
          acc[tt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[rr][cc][1], bf[s][0], acc[tt], 0, 0, 0);
          acc[tt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[rr][cc][0], bf[s][1], acc[tt], 0, 0, 0);
          acc[tt] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[rr][cc][0], bf[s][0], acc[tt], 0, 0, 0);
        }
      }
    }
  }

  const float inv = (sz_cur > 0.f) ? (1.f / sz_cur) * (1.f / sx_cur) : 0.f;
  float* slab = g.part + (size_t)split * g.Cout * 9 * g.Cin;
  const int c = c0 + 32 * wj + (lane & 31);
#pragma unroll
  for (int tt = 0; tt < NTAP; ++tt) {
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int n = n0 + 32 * wi + (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5);
      slab[((size_t)n * 9 + tt) * g.Cin + c] = acc[tt][reg] * inv;
    }
  }
  if (do_bias) {
    __syncthreads();  // the last tile's fragment reads are done before the LDS is reused
    float* rb = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int e = 0; e < 8; ++e) rb[tid * 8 + e] = bs[e];
    __syncthreads();
    if (tid < 64) {
      const int cg = tid >> 3, e = tid & 7;
      float sum = 0.f;
      for (int k = 0; k < NT / 8; ++k) sum += rb[(8 * k + cg) * 8 + e];
      g.part_bias[(size_t)split * g.Cout + n0 + tid] = sum;
    }
  }
}


// tile rows of the direct weight gradient: 4 (one block per CU) or 2 (pis_tune key 49: two per CU)
static int direct_w_rows() { return tune_get(PIS_TUNE_DIRECT_W_ROWS) == 2 ? 2 : WT_H; }

bool direct_w_wanted(int B, int H, int W, int Cin, int Cout, int ldx, int ldz) {
  if (!(B > 0 && H % WT_H == 0 && W % WT_W == 0 && Cin % 64 == 0 && Cout % 64 == 0 && ldz % 4 == 0 && ldx % 4 == 0))
    return false;
  return direct_h3_wanted(H, W, Cin, Cout, ldx);
}

// blocks: one per CU (4-row tiles) or two (2-row tiles), split over the (Cout, Cin) 64-blocks
static int direct_w_splits(int B, int H, int W, int Cin, int Cout) {
  const int rows = direct_w_rows(), target = rows == 2 ? 512 : 256;
  const int pairs = (Cout / 64) * (Cin / 64);
  const int ntile = B * (H / rows) * (W / WT_W);
  return std::max(1, std::min(ntile, target / std::max(1, std::min(pairs, target))));
}

size_t direct_w_ws_bytes(int B, int H, int W, int Cin, int Cout) {
  const int sp = direct_w_splits(B, H, W, Cin, Cout);
  return (size_t)sp * Cout * 9 * Cin * sizeof(float) + (size_t)sp * Cout * sizeof(float) + 512;
}

int reduce_slabs2(const float* part, int splits, int64_t n, float* dst, const float* part_b, int splits_b,
                  int64_t n_b, float* dst_b, int accumulate, hipStream_t s);

int launch_direct_wgrad(const float* x, int ldx, const float* dz, int ldz, float* dw, float* db, int B, int H, int W,
                        int Cin, int Cout, int acc, void* ws, size_t ws_bytes, hipStream_t s) {
  if (ws_bytes < direct_w_ws_bytes(B, H, W, Cin, Cout)) return set_error("direct wgrad: workspace too small"), PIS_ERR_ARG;
  DirectWArgs g{};
  g.x = x; g.ldx = ldx; g.dz = dz; g.ldz = ldz;
  g.B = B; g.H = H; g.W = W; g.Cin = Cin; g.Cout = Cout;
  g.splits = direct_w_splits(B, H, W, Cin, Cout);
  g.dbg = tune_get(PIS_TUNE_DEBUG_NOLOAD);
  g.vwalk = tune_get(PIS_TUNE_DIRECT_W_VWALK);
  g.part = reinterpret_cast<float*>(ws);
  g.part_bias = db ? g.part + (size_t)g.splits * Cout * 9 * Cin : nullptr;
  const int pairs = (Cout / 64) * (Cin / 64);
  const double flop = 2.0 * 9 * (double)B * H * W * Cin * Cout;
  const dim3 grid(g.splits * pairs);
  launch_hook("direct_wgrad_h3", 0, s, flop);
  if (g.dbg)
    hipLaunchKernelGGL((conv3x3_wgrad_h3_kernel<true>), grid, dim3(256), 0, s, g);
  else if (direct_w_rows() == 2)
    hipLaunchKernelGGL((conv3x3_wgrad_h3r_kernel<2>), grid, dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL((conv3x3_wgrad_h3_kernel<false>), grid, dim3(256), 0, s, g);
  launch_hook("direct_wgrad_h3", 1, s, flop);
  int rc = launch_status("conv3x3_wgrad_h3");
  // weights and bias in one launch (fixed-order sums, deterministic)
  if (!rc) rc = reduce_slabs2(g.part, g.splits, (int64_t)Cout * 9 * Cin, dw, g.part_bias, g.splits, Cout, db, acc, s);
  return rc;
}

}  // namespace pis
