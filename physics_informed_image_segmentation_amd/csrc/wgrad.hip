// Weight- and bias-gradient GEMMs (fp32 MFMA) for src/unet.py's 3x3 convs and
// 2x2 transposed convs, plus generic channel sums.
//
//   C[m'][n'] = sum_p A(p, m') * B(p, n')       p = pixel of the reduction grid
//   bias[m']  = sum_p A(p, m')                  (fused: blocks of the first n'-tile)
//
// The pixel reduction (up to B*H*W = 2.1M at 512^2) is split over blocks
// ("splits"); every block writes its partial C tile to a slab and a second
// kernel sums the slabs in a fixed order, so the result is deterministic and
// each fp32 accumulation chain is at most `pix_per_split` long. Logical block
// ids are XCD-remapped and split-major, so the tiles sharing one pixel range
// (e.g. the 9 taps of a conv) run on one XCD and re-read their inputs from
// that XCD's L2.
//
// conv3x3:  m' = n (Cout),        A(p, n)     = dz[p][n]
//           n' = (tap, c),        B(p, tap,c) = x[p + off(tap)][c]    (zero pad)
//           Cin == 1:  n' = tap (9 of 64 columns used)
// convT2x2: m' = (i, j, o),       A(p, ijo)   = dy[(2h+i, 2w+j)][o]
//           n' = c,               B(p, c)     = x[p][c]
#include "igemm.h"

namespace pis {

enum BMode { B_PLAIN = 0, B_CONV3 = 1, B_CONV3_C1 = 2 };

struct WgradArgs {
  const float* a; int lda; int a_up2; int Ca;   // Ca: channels per (i,j) group when a_up2
  const float* b; int ldb; int b_mode; int Cb;   // Cb: channels per tap when B_CONV3
  int B, H, W;                                   // reduction pixel grid
  int P;                                         // B*H*W
  int Mp, Np;                                    // output dims (Np padded for B_CONV3_C1)
  int pix_per_split;
  float* part;                                   // [splits][Mp][Np]
  float* part_bias;                              // [splits][Mp] or NULL
  // batched launches (gridDim.y > 1, Winograd's 16 GEMMs): per-batch offsets; slab pitch
  int64_t bs_a, bs_b, bs_part, split_stride;     // split_stride 0 = Mp * Np
  int pair;                                      // wgrad_x6: pair-lane staging of 4-pixel operands
  int bias_xi;                                   // batched launches: the batch whose column sums of A are
                                                 // the bias partials (Winograd: 7, E's (1, 1) plane; 0 when
                                                 // the launch has one batch)
  int dbg;                                       // wgrad_h3t timing twins (pis_tune key 2, wrong results):
                                                 // 1 no loads after the first two K-steps, 2 no staging
                                                 // after the first, 4 no slab stores
};

// BKP pixels per stage: 32 MFMAs per wave between barriers for every tile shape
template <int BM, int BN, int BKP>
__global__ __launch_bounds__(256) void wgrad_f32_kernel(WgradArgs g) {
  const Remap2 rm = xcd_remap2();
  if (rm.batch) {
    g.a += rm.batch * g.bs_a;
    g.b += rm.batch * g.bs_b;
    g.part += rm.batch * g.bs_part;
  }
  constexpr int TM = BM / 64, TN = BN / 64;   // 32x32 tiles per wave
  constexpr int AL = BKP * BM / 4 / 256, BL = BKP * BN / 4 / 256;
  __shared__ __attribute__((aligned(16))) float sA[2][BKP * BM];
  __shared__ __attribute__((aligned(16))) float sB[2][BKP * BN];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntm = g.Mp / BM, ntn = g.Np / BN;
  const int tiles = ntm * ntn;
  const int bid = rm.bid;
  const int split = bid / tiles;
  const int tile = bid - split * tiles;
  const int tm = tile / ntn, tn = tile % ntn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int p_begin = split * g.pix_per_split;
  const int p_end = min(g.P, p_begin + g.pix_per_split);
  const bool do_bias = g.part_bias != nullptr && tn == 0 && rm.batch == g.bias_xi;

  // tap of this tile (tiles never straddle a tap)
  int a_dr = 0, a_ds = 0, a_c0 = m0;
  if (g.a_up2) { const int ij = m0 / g.Ca; a_dr = ij >> 1; a_ds = ij & 1; a_c0 = m0 - ij * g.Ca; }
  int b_dr = 0, b_ds = 0, b_c0 = n0;
  if (g.b_mode == B_CONV3) { const int t = n0 / g.Cb; b_dr = t / 3 - 1; b_ds = t % 3 - 1; b_c0 = n0 - t * g.Cb; }
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
      if (p >= p_end) continue;
      if (g.b_mode == B_PLAIN) {
        rb[i] = *reinterpret_cast<const f32x4*>(g.b + (size_t)p * g.ldb + b_c0 + c);
      } else {
        const int bb = p / HW, rem = p - bb * HW, h = rem / g.W, w = rem - h * g.W;
        if (g.b_mode == B_CONV3) {
          const int hs = h + b_dr, ws = w + b_ds;
          if (hs >= 0 && hs < g.H && ws >= 0 && ws < g.W)
            rb[i] = *reinterpret_cast<const f32x4*>(g.b + (((size_t)bb * g.H + hs) * g.W + ws) * g.ldb + b_c0 + c);
        } else {  // B_CONV3_C1: columns are taps 0..8 of a single input channel
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int t = n0 + c + j;
            if (t < 9) {
              const int hs = h + t / 3 - 1, ws = w + t % 3 - 1;
              if (hs >= 0 && hs < g.H && ws >= 0 && ws < g.W)
                rb[i][j] = g.b[(((size_t)bb * g.H + hs) * g.W + ws) * g.ldb];
            }
          }
        }
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
  float bsum = 0.f;

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
    if (do_bias && tid < BM) {
#pragma unroll
      for (int r = 0; r < BKP; ++r) bsum += As[r * BM + tid];
    }
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

  float* out = g.part + (size_t)split * (g.split_stride ? g.split_stride : (int64_t)g.Mp * g.Np);
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
  if (do_bias && tid < BM) g.part_bias[(size_t)split * g.Mp + m0 + tid] = bsum;
}

// ---------------------------------------------------------------------------
// conv3x3 weight gradient, all 9 taps per block from one staged halo.
//
// Block tile: 64 output channels (m0) x 64 input channels (c0) x 9 taps; the
// four waves own the (32-row, 32-col) quadrants, each with 9 accumulators (one
// per tap, 144 AGPRs). The pixel reduction walks 16-pixel segments of image
// rows: per stage the block stages dz[16 px][64] and the three input rows
// h-1..h+1, columns w0-1..w0+16 ([3][18][64], zero padded) once, and every
// tap reads its shifted window from LDS. 72 MFMAs per wave per barrier; each
// input element is fetched 3x per block (once per kernel row) instead of 9x.
// ---------------------------------------------------------------------------
struct W3Args {
  const float* x; int ldx;
  const float* dz; int ldz;
  int B, H, W, Cin, Cout;
  int seg_per_split;   // 16-pixel row segments per split
  int nseg;            // B*H*W/16
  float* part;         // [splits][Cout][9][Cin]
  float* part_bias;    // [splits][Cout] or NULL
};

// NSEG consecutive 16-pixel segments per stage (one barrier per NSEG * 72 MFMAs).
template <int NSEG>
__global__ __launch_bounds__(256, 2) void wgrad3x3_halo_kernel(W3Args g) {
  constexpr int SEG = 16, HW_ = SEG + 2, CH = 64;
  constexpr int X_F4 = 3 * HW_ * CH / 4;          // 864 float4 of halo per segment
  constexpr int XS = 3 * HW_ * CH;                 // floats of halo per segment
  constexpr int XL = (NSEG * X_F4 + 255) / 256;    // float4 loads per thread per stage
  __shared__ __attribute__((aligned(16))) float sD[2][NSEG * SEG * CH];
  __shared__ __attribute__((aligned(16))) float sX[2][NSEG * XS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int ntc = g.Cin / CH, ntm = g.Cout / CH;
  const int tiles = ntc * ntm;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int split = bid / tiles;
  const int tile = bid - split * tiles;
  const int m0 = (tile / ntc) * CH, c0 = (tile % ntc) * CH;
  const int s_begin = split * g.seg_per_split;
  const int s_end = min(g.nseg, s_begin + g.seg_per_split);
  const bool do_bias = g.part_bias != nullptr && c0 == 0;
  const int segs_per_row = g.W / SEG;

  f32x4 rd[NSEG], rx[XL];
  auto gload = [&](int sg0) {
    int sb[NSEG], sh[NSEG], sw[NSEG];
    bool sv[NSEG];
#pragma unroll
    for (int j = 0; j < NSEG; ++j) {  // block-uniform segment coordinates
      const int sg = sg0 + j;
      sv[j] = sg < s_end;
      const int row_id = sg / segs_per_row;  // b*H + h
      sw[j] = (sg - row_id * segs_per_row) * SEG;
      sb[j] = row_id / g.H;
      sh[j] = row_id - sb[j] * g.H;
      const int px = tid >> 4, c4 = (tid & 15) * 4;
      rd[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (sv[j])
        rd[j] = *reinterpret_cast<const f32x4*>(g.dz + ((size_t)row_id * g.W + sw[j] + px) * g.ldz + m0 + c4);
    }
#pragma unroll
    for (int i = 0; i < XL; ++i) {
      const int idx = tid + i * 256;
      rx[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (idx < NSEG * X_F4) {
        const int j = NSEG == 1 ? 0 : idx / X_F4;
        const int e = idx - j * X_F4;
        const int r = e / (HW_ * 16), rem = e - r * (HW_ * 16);
        const int px = rem >> 4, c4 = (rem & 15) * 4;
        const int b = NSEG == 1 ? sb[0] : (j ? sb[NSEG - 1] : sb[0]);
        const int h = NSEG == 1 ? sh[0] : (j ? sh[NSEG - 1] : sh[0]);
        const int w0 = NSEG == 1 ? sw[0] : (j ? sw[NSEG - 1] : sw[0]);
        const bool v = NSEG == 1 ? sv[0] : (j ? sv[NSEG - 1] : sv[0]);
        const int hs = h + r - 1, ws = w0 + px - 1;
        if (v && hs >= 0 && hs < g.H && ws >= 0 && ws < g.W)
          rx[i] = *reinterpret_cast<const f32x4*>(g.x + (((size_t)b * g.H + hs) * g.W + ws) * g.ldx + c0 + c4);
      }
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int j = 0; j < NSEG; ++j) *reinterpret_cast<f32x4*>(&sD[buf][j * SEG * CH + tid * 4]) = rd[j];
#pragma unroll
    for (int i = 0; i < XL; ++i) {
      const int idx = tid + i * 256;
      if (idx < NSEG * X_F4) *reinterpret_cast<f32x4*>(&sX[buf][idx * 4]) = rx[i];
    }
  };

  f32x16 acc[9];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
  float bsum = 0.f;
  const int li = lane & 31, lh = lane >> 5;
  const int nst = (s_end - s_begin + NSEG - 1) / NSEG;
  if (nst > 0) {
    gload(s_begin);
    lstore(0);
  }
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    if (st + 1 < nst) gload(s_begin + (st + 1) * NSEG);
    const float* D = sD[cur];
    const float* X = sX[cur];
    if (do_bias && tid < CH) {
#pragma unroll
      for (int r = 0; r < NSEG * SEG; ++r) bsum += D[r * CH + tid];
    }
#pragma unroll
    for (int kk = 0; kk < NSEG * SEG / 2; ++kk) {
      const int j = kk / (SEG / 2);
      const int px = 2 * (kk - j * (SEG / 2)) + lh;  // pixel within segment j
      const float a = D[(j * SEG + px) * CH + wm * 32 + li];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int r = t / 3, s = t % 3;  // x at (h + r - 1, w + s - 1) = halo (r, px + s)
        const float bv = X[j * XS + (r * HW_ + px + s) * CH + wn * 32 + li];
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv, acc[t], 0, 0, 0);
      }
    }
    if (st + 1 < nst) lstore(cur ^ 1);
    __syncthreads();
  }
  float* out = g.part + (size_t)split * g.Cout * 9 * g.Cin;
  const int c = c0 + wn * 32 + li;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int n = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
      out[((size_t)n * 9 + t) * g.Cin + c] = acc[t][r];
    }
  if (do_bias && tid < CH) g.part_bias[(size_t)split * g.Cout + m0 + tid] = bsum;
}

// dst[i] = (acc ? dst[i] : 0) + sum_s part[s*pitch + i]: every thread sums the
// slabs of its residue class (fixed order), then a fixed LDS tree: deterministic.
template <int VEC>
__global__ __launch_bounds__(256) void reduce_slabs_kernel(const float* __restrict__ part, int splits,
                                                           int64_t n, int64_t pitch,
                                                           float* __restrict__ dst, int accumulate,
                                                           int cols) {
  typedef float vec __attribute__((ext_vector_type(VEC)));
  const int groups = 256 / cols;
  const int gi = threadIdx.x / cols, c = threadIdx.x - gi * cols;
  const int64_t nv = n / VEC;
  const int64_t col = (int64_t)blockIdx.x * cols + c;
  vec s = (vec)(0.f);
  if (col < nv) {
    // 8 independent partial sums keep 8 loads in flight per thread; combined in a fixed order
    vec s8[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) s8[u] = (vec)(0.f);
    int k = gi;
    for (; k + 7 * groups < splits; k += 8 * groups) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
        s8[u] += *reinterpret_cast<const vec*>(part + (size_t)(k + u * groups) * pitch + col * VEC);
    }
    for (int u = 0; k < splits; k += groups, ++u)
      s8[u & 7] += *reinterpret_cast<const vec*>(part + (size_t)k * pitch + col * VEC);
#pragma unroll
    for (int u = 0; u < 8; ++u) s += s8[u];
  }
  __shared__ vec red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  // fixed-order pairwise tree over the groups (deterministic; log2(groups) barrier steps)
  for (int stride = groups / 2; stride >= 1; stride /= 2) {
    if (gi < stride) red[gi * cols + c] += red[(gi + stride) * cols + c];
    __syncthreads();
  }
  if (gi == 0 && col < nv) {
    vec t = accumulate ? *reinterpret_cast<vec*>(dst + col * VEC) : (vec)(0.f);
    *reinterpret_cast<vec*>(dst + col * VEC) = t + red[c];
  }
}

int reduce_slabs_pitched(const float* part, int splits, int64_t n, int64_t pitch, float* dst,
                         int accumulate, hipStream_t s) {
  const bool v4 = (n % 4 == 0) && (pitch % 4 == 0) && ((uintptr_t)part % 16 == 0) && ((uintptr_t)dst % 16 == 0);
  const int64_t nv = v4 ? n / 4 : n;
  // threads per column-block: up to 64 slab groups for many slabs, narrower blocks for small outputs
  // thousands of slabs over a few columns (the bias partials of the dz transforms): all 256
  // threads of a block walk slabs, so the per-thread chains stay short
  const int gmax = splits >= 1024 ? 256 : 64;
  int gwant = 1;
  while (gwant < gmax && gwant < splits) gwant *= 2;
  int cols = std::max(splits >= 1024 ? 1 : 4, 256 / gwant);
  while (cols > 1 && cols / 2 >= nv) cols /= 2;
  const int grid = (int)cdiv(nv, cols);
  if (v4)
    hipLaunchKernelGGL(reduce_slabs_kernel<4>, dim3(grid), dim3(256), 0, s, part, splits, n, pitch, dst,
                       accumulate, cols);
  else
    hipLaunchKernelGGL(reduce_slabs_kernel<1>, dim3(grid), dim3(256), 0, s, part, splits, n, pitch, dst,
                       accumulate, cols);
  return launch_status("reduce_slabs");
}

// Thousands of slabs over a few columns (the per-block bias partials of the dz transforms: 8192
// slabs x 64 channels at 512^2): pass 1 lets block g sum a contiguous chunk of slabs with
// coalesced row reads (n/4 float4 lanes per row, 256/(n/4) rows in flight) and writes its sum
// over the FIRST slab of its own chunk (which only it reads); pass 2 is the pitched reduction of
// those G rows. Both orders are fixed: deterministic. (One column per block across all slabs
// fetched each 128-B line once per float4 column: 30-50 us per bias at 512^2.)
__global__ __launch_bounds__(256) void reduce_rows_chunk_kernel(float* __restrict__ part, int splits, int n4,
                                                                int chunk) {
  const int R = 256 / n4, r = threadIdx.x / n4, c = threadIdx.x - r * n4;
  const int s0 = blockIdx.x * chunk, s1 = min(splits, s0 + chunk);
  const int64_t n = 4 * (int64_t)n4;
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;  // four chains: loads in flight
  if (r < R) {
    int k = s0 + r;
    for (; k + 3 * R < s1; k += 4 * R) {
      a0 += *reinterpret_cast<const f32x4*>(part + (int64_t)k * n + 4 * c);
      a1 += *reinterpret_cast<const f32x4*>(part + (int64_t)(k + R) * n + 4 * c);
      a2 += *reinterpret_cast<const f32x4*>(part + (int64_t)(k + 2 * R) * n + 4 * c);
      a3 += *reinterpret_cast<const f32x4*>(part + (int64_t)(k + 3 * R) * n + 4 * c);
    }
    if (k < s1) a0 += *reinterpret_cast<const f32x4*>(part + (int64_t)k * n + 4 * c);
    if (k + R < s1) a1 += *reinterpret_cast<const f32x4*>(part + (int64_t)(k + R) * n + 4 * c);
    if (k + 2 * R < s1) a2 += *reinterpret_cast<const f32x4*>(part + (int64_t)(k + 2 * R) * n + 4 * c);
  }
  __shared__ f32x4 red[256];
  red[threadIdx.x] = (a0 + a1) + (a2 + a3);
  __syncthreads();  // every read of this chunk is done before its first slab is overwritten
  if (r == 0) {
    f32x4 t = red[c];
    for (int q = 1; q < R; ++q) t += red[q * n4 + c];
    *reinterpret_cast<f32x4*>(part + (int64_t)s0 * n + 4 * c) = t;
  }
}

// Two slab reductions in ONE launch (a weight gradient's [split][n] slabs and its bias gradient's
// [split][Cout] partials): the blocks of the second follow the first's; each block runs
// reduce_slabs_kernel's fixed-order sums on its own job (float4 or scalar columns per job). Same
// sums in the same order as two reduce_slabs_pitched launches: bitwise equal, one launch fewer.
struct SlabJob {
  const float* part;
  float* dst;
  int64_t n, pitch;
  int splits, accumulate;
  int vec, cols, blocks;  // launch plan (slab_job_plan)
};

static SlabJob slab_job_plan(const float* part, int splits, int64_t n, int64_t pitch, float* dst, int accumulate) {
  SlabJob j{part, dst, n, pitch, splits, accumulate, 1, 1, 0};
  const bool v4 = (n % 4 == 0) && (pitch % 4 == 0) && ((uintptr_t)part % 16 == 0) && ((uintptr_t)dst % 16 == 0);
  j.vec = v4 ? 4 : 1;
  const int64_t nv = n / j.vec;
  const int gmax = splits >= 1024 ? 256 : 64;  // as reduce_slabs_pitched
  int gwant = 1;
  while (gwant < gmax && gwant < splits) gwant *= 2;
  int cols = std::max(splits >= 1024 ? 1 : 4, 256 / gwant);
  while (cols > 1 && cols / 2 >= nv) cols /= 2;
  j.cols = cols;
  j.blocks = (int)cdiv(nv, cols);
  return j;
}

template <int VEC>
__device__ __forceinline__ void reduce_slab_job(const SlabJob& j, int blk) {
  typedef float vec __attribute__((ext_vector_type(VEC)));
  const int cols = j.cols, groups = 256 / cols;
  const int gi = threadIdx.x / cols, c = threadIdx.x - gi * cols;
  const int64_t nv = j.n / VEC;
  const int64_t col = (int64_t)blk * cols + c;
  vec s = (vec)(0.f);
  if (col < nv) {
    vec s8[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) s8[u] = (vec)(0.f);
    int k = gi;
    for (; k + 7 * groups < j.splits; k += 8 * groups) {
#pragma unroll
      for (int u = 0; u < 8; ++u)
        s8[u] += *reinterpret_cast<const vec*>(j.part + (size_t)(k + u * groups) * j.pitch + col * VEC);
    }
    for (int u = 0; k < j.splits; k += groups, ++u)
      s8[u & 7] += *reinterpret_cast<const vec*>(j.part + (size_t)k * j.pitch + col * VEC);
#pragma unroll
    for (int u = 0; u < 8; ++u) s += s8[u];
  }
  __shared__ vec red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int stride = groups / 2; stride >= 1; stride /= 2) {
    if (gi < stride) red[gi * cols + c] += red[(gi + stride) * cols + c];
    __syncthreads();
  }
  if (gi == 0 && col < nv) {
    vec t = j.accumulate ? *reinterpret_cast<vec*>(j.dst + col * VEC) : (vec)(0.f);
    *reinterpret_cast<vec*>(j.dst + col * VEC) = t + red[c];
  }
}

__global__ __launch_bounds__(256) void reduce_slabs2_kernel(SlabJob a, SlabJob b) {
  const bool first = (int)blockIdx.x < a.blocks;
  const SlabJob& j = first ? a : b;
  const int blk = first ? (int)blockIdx.x : (int)blockIdx.x - a.blocks;
  if (j.vec == 4) reduce_slab_job<4>(j, blk);
  else reduce_slab_job<1>(j, blk);
}

int reduce_slabs(const float* part, int splits, int64_t n, float* dst, int accumulate, hipStream_t s);

// reduce_slabs' chunked two-pass regime (many slabs of a short row, PIS_TUNE_SLAB_CHUNKS)
static bool slabs_chunked(const float* part, int splits, int64_t n, const float* dst) {
  const bool v4 = (n % 4 == 0) && ((uintptr_t)part % 16 == 0) && ((uintptr_t)dst % 16 == 0);
  return v4 && splits >= 1024 && n <= 1024 && tune_get(PIS_TUNE_SLAB_CHUNKS) != 0;
}

// the two reductions of a weight gradient (weights, then bias) in one launch. A weights-only call
// (bias NULL) is reduce_slabs itself, chunked regime (key 20) included. A weights + bias pair is
// always the merged single-pass launch, whatever key 20 says: the pair's extra launches of the
// chunked form cost more than the merged launch saves on the few pairs in that regime (round 5's
// reduction glue, 53 -> 14 launches per step). NOTE: like reduce_slabs, may overwrite part.
int reduce_slabs2(const float* part, int splits, int64_t n, float* dst, const float* part_b, int splits_b,
                  int64_t n_b, float* dst_b, int accumulate, hipStream_t s) {
  if (!dst_b) return reduce_slabs(part, splits, n, dst, accumulate, s);
  const SlabJob a = slab_job_plan(part, splits, n, n, dst, accumulate);
  const SlabJob b = slab_job_plan(part_b, splits_b, n_b, n_b, dst_b, accumulate);
  hipLaunchKernelGGL(reduce_slabs2_kernel, dim3(a.blocks + b.blocks), dim3(256), 0, s, a, b);
  return launch_status("reduce_slabs2");
}

// NOTE: may overwrite part (every caller passes its own partial-slab scratch)
int reduce_slabs(const float* part, int splits, int64_t n, float* dst, int accumulate, hipStream_t s) {
  if (slabs_chunked(part, splits, n, dst)) {
    const int G = std::min(256, splits / 16);
    const int chunk = (int)cdiv(splits, G), nblk = (int)cdiv(splits, chunk);
    hipLaunchKernelGGL(reduce_rows_chunk_kernel, dim3(nblk), dim3(256), 0, s, const_cast<float*>(part), splits,
                       (int)(n / 4), chunk);
    const int rc = launch_status("reduce_rows_chunk");
    if (rc) return rc;
    return reduce_slabs_pitched(part, nblk, n, (int64_t)chunk * n, dst, accumulate, s);
  }
  return reduce_slabs_pitched(part, splits, n, n, dst, accumulate, s);
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
  if (r < rows) {
    // 4 independent partial sums keep 4 loads in flight per thread (fixed combine order)
    f32x4 s4[4] = {s, s, s, s};
    int64_t p = p0 + r;
    for (; p + 3 * rows < p1; p += 4 * rows) {
#pragma unroll
      for (int u = 0; u < 4; ++u) s4[u] += *reinterpret_cast<const f32x4*>(src + (p + u * rows) * ld + 4 * c4);
    }
    for (int u = 0; p < p1; p += rows, ++u) s4[u & 3] += *reinterpret_cast<const f32x4*>(src + p * ld + 4 * c4);
    s = (s4[0] + s4[1]) + (s4[2] + s4[3]);
  }
  __shared__ f32x4 red[256];
  red[tid] = s;
  __syncthreads();
  if (tid < c4n) {
    f32x4 t = red[tid];
    for (int k = 1; k < rows; ++k) t += red[k * c4n + tid];
    *reinterpret_cast<f32x4*>(part + (size_t)blockIdx.x * C + 4 * tid) = t;
  }
}

// Scalar column sum for C not a multiple of 4: one sum per block and channel
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
  // ~1024 blocks (4 per CU) whatever the size: the pass is one read of the source
  pps = std::max<int64_t>(64, cdiv(npix, 1024));
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
  size_t part_bytes, bias_bytes;
};

static WgradPlan plan_wgrad(int Mp, int Np, int P, int group_m, int group_n, int target_blocks = 2048) {
  // tile sizes must divide the per-tap group so tiles never straddle a tap
  WgradPlan p{};
  p.bm = (Mp % 128 == 0 && group_m % 128 == 0) ? 128 : 64;
  p.bn = (Np % 128 == 0 && group_n % 128 == 0) ? 128 : 64;
  const int tiles = (Mp / p.bm) * (Np / p.bn);
  // >= ~2 blocks per CU, fp32 chains of at most 8192 pixels, at least 64 pixels per split
  // >= ~8 blocks per CU so the tail wave is short; partial-slab traffic stays
  // ~2 bytes per 1000 FLOP at >= 512 pixels per split
  const int64_t want_splits = std::max<int64_t>(1, cdiv(target_blocks, tiles));
  int64_t pps = std::max<int64_t>(512, cdiv(P, want_splits));
  pps = std::min<int64_t>(pps, 8192);
  pps = cdiv(pps, 64) * 64;
  p.pps = (int)pps;
  p.splits = (int)cdiv(P, pps);
  p.part_bytes = (size_t)p.splits * Mp * Np * sizeof(float);
  p.bias_bytes = (size_t)p.splits * Mp * sizeof(float);
  return p;
}

// part slabs at ws, bias slabs right after them (16-byte aligned)
static float* bias_slabs(void* ws, const WgradPlan& pl) {
  return (float*)((char*)ws + cdiv(pl.part_bytes, 256) * 256);
}

static size_t wgrad_ws_bytes(const WgradPlan& pl) { return cdiv(pl.part_bytes, 256) * 256 + pl.bias_bytes + 256; }

// The same split-K contraction at fp32 accuracy on bf16 MFMA (bf16x6, as gemm_nt_x6_kernel in
// winograd.hip) for plain row operands B (the Winograd weight gradient: A = E[t][Cout],
// B = V[t][Cin]). The pixel (K) axis is the row index in memory, so each thread
// loads one column (m or n) over 8 (or 4) consecutive pixels with coalesced scalar loads and
// writes the three bf16 planes K-contiguous ([m][16 k], one 16-B / 8-B LDS store per plane):
// the MFMA operand fragment (8 consecutive k of one row) is then a single ds_read_b128.
// Also the transposed-conv weight gradient (a_up2 rows, bias column sums of A).
typedef __bf16 wbf16x8 __attribute__((ext_vector_type(8)));

template <int E>  // E = 8 or 4 consecutive-k values of one row -> one 16-B / 8-B store per plane
__device__ __forceinline__ void wsplit_store(const float (&v)[E], __bf16* p0, __bf16* p1, __bf16* p2) {
  u32x2 h0, m0, l0;
  split3_x4(f32x4{v[0], v[1], v[2], v[3]}, h0, m0, l0);
  if constexpr (E == 8) {
    u32x2 h1, m1, l1;
    split3_x4(f32x4{v[4], v[5], v[6], v[7]}, h1, m1, l1);
    *reinterpret_cast<u32x4*>(p0) = u32x4{h0[0], h0[1], h1[0], h1[1]};
    *reinterpret_cast<u32x4*>(p1) = u32x4{m0[0], m0[1], m1[0], m1[1]};
    *reinterpret_cast<u32x4*>(p2) = u32x4{l0[0], l0[1], l1[0], l1[1]};
  } else {
    *reinterpret_cast<u32x2*>(p0) = h0;
    *reinterpret_cast<u32x2*>(p1) = m0;
    *reinterpret_cast<u32x2*>(p2) = l0;
  }
}

template <int BM, int BN>
__global__ __launch_bounds__(256, 2) void wgrad_x6_kernel(WgradArgs g) {
  const Remap2 rm = xcd_remap2();
  if (rm.batch) {
    g.a += rm.batch * g.bs_a;
    g.b += rm.batch * g.bs_b;
    g.part += rm.batch * g.bs_part;
  }
  constexpr int BK = 16;
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int EA = BM * BK / 256, EB = BN * BK / 256;  // pixels per thread per stage (8 or 4)
  __shared__ __attribute__((aligned(16))) __bf16 sA[2][3][BM * BK];  // [buf][hi|mid|lo][m][k]
  __shared__ __attribute__((aligned(16))) __bf16 sB[2][3][BN * BK];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, lh = lane >> 5;
  const int ntm = g.Mp / BM, ntn = g.Np / BN;
  const int tiles = ntm * ntn;
  const int bid = rm.bid;
  const int split = bid / tiles;
  const int tile = bid - split * tiles;
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const int p_begin = split * g.pix_per_split;
  const int p_end = min(g.P, p_begin + g.pix_per_split);
  // this thread's column and pixel offset. g.pair (pis_tune 21, off by default): with 4 pixels
  // per thread (64-wide tiles) the two lanes of a pair take the two 8-B halves of one 16-B chunk
  // of one row, so a ds_write_b64 lane group covers 8 rows x 16 B: with the row swizzle, 16
  // distinct 8-B slots (one pixel group per lane: 2-way conflicts, but better-coalesced loads)
  const bool pa = EA == 4 && g.pair, pb = EB == 4 && g.pair;
  const int am = pa ? (tid >> 1) % BM : tid % BM;
  const int ap = pa ? 8 * (tid / (2 * BM)) + 4 * (tid & 1) : (tid / BM) * EA;
  const int bn = pb ? (tid >> 1) % BN : tid % BN;
  const int bp = pb ? 8 * (tid / (2 * BN)) + 4 * (tid & 1) : (tid / BN) * EB;
  const bool do_bias = g.part_bias != nullptr && n0 == 0 && rm.batch == g.bias_xi;
  // a_up2 (transposed-conv weight gradient): the tile's (i, j) tap of the 2x2 output block
  int a_dr = 0, a_ds = 0, a_c0 = m0;
  if (g.a_up2) { const int ij = m0 / g.Ca; a_dr = ij >> 1; a_ds = ij & 1; a_c0 = m0 - ij * g.Ca; }
  const int HW = g.H * g.W;
  float ra[EA], rb[EB];
  float bsum = 0.f;
  auto gload = [&](int p0) {
    // a_up2: the EA pixels sit in one image row (W % EA == 0, checked by the launcher), two
    // output pixels apart
    size_t pix0 = p0 + ap;
    int pstep = 1;
    if (g.a_up2) {
      const int p = p0 + ap;
      const int bb = p / HW, rem = p - bb * HW, h = rem / g.W, w = rem - h * g.W;
      pix0 = ((size_t)bb * 2 * g.H + 2 * h + a_dr) * (2 * g.W) + 2 * w + a_ds;
      pstep = 2;
    }
#pragma unroll
    for (int e = 0; e < EA; ++e) {
      const int p = p0 + ap + e;
      ra[e] = p < p_end ? g.a[(pix0 + (size_t)pstep * e) * g.lda + a_c0 + am] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const int p = p0 + bp + e;
      rb[e] = p < p_end ? g.b[(size_t)p * g.ldb + n0 + bn] : 0.f;
    }
  };
  auto lstore = [&](int buf) {
    if (do_bias) {
#pragma unroll
      for (int e = 0; e < EA; ++e) bsum += ra[e];
    }
    wsplit_store<EA>(ra, &sA[buf][0][wsw(am, ap)], &sA[buf][1][wsw(am, ap)], &sA[buf][2][wsw(am, ap)]);
    wsplit_store<EB>(rb, &sB[buf][0][wsw(bn, bp)], &sB[buf][1][wsw(bn, bp)], &sB[buf][2][wsw(bn, bp)]);
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const int nst = (p_end - p_begin + BK - 1) / BK;
  if (nst > 0) {
    gload(p_begin);
    lstore(0);
  }
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    if (st + 1 < nst) gload(p_begin + (st + 1) * BK);
    wbf16x8 af[3][TM], bf[3][TN];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
#pragma unroll
      for (int a = 0; a < TM; ++a)
        af[pl][a] = *reinterpret_cast<const wbf16x8*>(&sA[cur][pl][wsw(wm * (BM / 2) + a * 32 + li, 8 * lh)]);
#pragma unroll
      for (int b = 0; b < TN; ++b)
        bf[pl][b] = *reinterpret_cast<const wbf16x8*>(&sB[cur][pl][wsw(wn * (BN / 2) + b * 32 + li, 8 * lh)]);
    }
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {  // smallest partial products first
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2][a], bf[0][b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][a], bf[1][b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][a], bf[2][b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][a], bf[0][b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][a], bf[1][b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][a], bf[0][b], acc[a][b], 0, 0, 0);
      }
    if (st + 1 < nst) lstore(cur ^ 1);
    __syncthreads();
  }
  float* out = g.part + (size_t)split * (g.split_stride ? g.split_stride : (int64_t)g.Mp * g.Np);
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
  if (do_bias) {  // column sums of A: 256 / BM partial sums per column, reduced through LDS
    float* red = reinterpret_cast<float*>(&sA[0][0][0]);
    red[tid] = bsum;
    __syncthreads();
    if (tid < BM) {  // the threads whose column am is tid, in a fixed order
      float t = 0.f;
      if (!pa) {
#pragma unroll
        for (int q = 0; q < 256 / BM; ++q) t += red[q * BM + tid];
      } else {
#pragma unroll
        for (int q = 0; q < 256 / (2 * BM); ++q) t += red[q * 2 * BM + 2 * tid] + red[q * 2 * BM + 2 * tid + 1];
      }
      g.part_bias[(size_t)split * g.Mp + m0 + tid] = t;
    }
  }
}

// The same contraction in fp16x3 (common.h): hi/lo fp16 planes, three fp16 MFMA
// products, per-wave per-K-step power-of-two scales. The TPR = 16 / E threads that stage one
// row's 16 pixels of a K-step are consecutive lanes of ONE wave (row = tid / TPR), so a row is
// scaled uniformly; row m of the tile was staged by wave m / (64 / TPR). Accumulator register r
// of block (a, b) is in units sA[wave of its row] * sB[wave of its column].
template <int BM, int BN>
__global__ __launch_bounds__(256, 2) void wgrad_h3_kernel(WgradArgs g) {
  const Remap2 rm = xcd_remap2();
  if (rm.batch) {
    g.a += rm.batch * g.bs_a;
    g.b += rm.batch * g.bs_b;
    g.part += rm.batch * g.bs_part;
  }
  constexpr int BK = 16;
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int EA = BM * BK / 256, EB = BN * BK / 256;  // pixels per thread per stage (8 or 4)
  constexpr int TPA = BK / EA, TPB = BK / EB;            // threads per row
  constexpr int RWA = 64 / TPA, RWB = 64 / TPB;          // rows staged per wave
  __shared__ __attribute__((aligned(16))) _Float16 sA[2][2][BM * BK];  // [buf][hi|lo][m][k]
  __shared__ __attribute__((aligned(16))) _Float16 sB[2][2][BN * BK];
  __shared__ __attribute__((aligned(16))) float sscale[2][2][4];      // [buf][A|B][staging wave]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, lh = lane >> 5;
  const int ntm = g.Mp / BM, ntn = g.Np / BN;
  const int tiles = ntm * ntn;
  const int bid = rm.bid;
  const int split = bid / tiles;
  const int tile = bid - split * tiles;
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const int p_begin = split * g.pix_per_split;
  const int p_end = min(g.P, p_begin + g.pix_per_split);
  const int am = tid / TPA, ap = (tid % TPA) * EA;
  const int bn = tid / TPB, bp = (tid % TPB) * EB;
  const bool do_bias = g.part_bias != nullptr && n0 == 0 && rm.batch == g.bias_xi;
  int a_dr = 0, a_ds = 0, a_c0 = m0;
  if (g.a_up2) { const int ij = m0 / g.Ca; a_dr = ij >> 1; a_ds = ij & 1; a_c0 = m0 - ij * g.Ca; }
  const int HW = g.H * g.W;
  float ra[EA], rb[EB];
  float bsum = 0.f;
  auto gload = [&](int p0) {
    size_t pix0 = p0 + ap;
    int pstep = 1;
    if (g.a_up2) {
      const int p = p0 + ap;
      const int bb = p / HW, rem = p - bb * HW, h = rem / g.W, w = rem - h * g.W;
      pix0 = ((size_t)bb * 2 * g.H + 2 * h + a_dr) * (2 * g.W) + 2 * w + a_ds;
      pstep = 2;
    }
#pragma unroll
    for (int e = 0; e < EA; ++e) {
      const int p = p0 + ap + e;
      ra[e] = p < p_end ? g.a[(pix0 + (size_t)pstep * e) * g.lda + a_c0 + am] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < EB; ++e) {
      const int p = p0 + bp + e;
      rb[e] = p < p_end ? g.b[(size_t)p * g.ldb + n0 + bn] : 0.f;
    }
  };
  float sa = 0.f, sb = 0.f;  // this wave's current scales (h3_keep)
  float sa_min = __builtin_inff(), sb_min = __builtin_inff();  // ... and the smallest so far
  auto store_row = [&](const float* v, int E, float sc, _Float16* hp, _Float16* lp) {
    u32x2 h0, l0;
    split2h_x4(f32x4{v[0], v[1], v[2], v[3]} * sc, h0, l0);
    if (E == 8) {
      u32x2 h1, l1;
      split2h_x4(f32x4{v[4], v[5], v[6], v[7]} * sc, h1, l1);
      *reinterpret_cast<u32x4*>(hp) = u32x4{h0[0], h0[1], h1[0], h1[1]};
      *reinterpret_cast<u32x4*>(lp) = u32x4{l0[0], l0[1], l1[0], l1[1]};
    } else {
      *reinterpret_cast<u32x2*>(hp) = h0;
      *reinterpret_cast<u32x2*>(lp) = l0;
    }
  };
  auto lstore = [&](int buf) {
    float ma = 0.f, mb = 0.f;
#pragma unroll
    for (int e = 0; e < EA; ++e) {
      if (do_bias) bsum += ra[e];
      ma = fmaxf(ma, fabsf(ra[e]));
    }
#pragma unroll
    for (int e = 0; e < EB; ++e) mb = fmaxf(mb, fabsf(rb[e]));
    sa = h3_keep(sa, wave_max_nonneg(ma), sa_min);
    sb = h3_keep(sb, wave_max_nonneg(mb), sb_min);
    if (lane == 0) {
      sscale[buf][0][wave] = sa;
      sscale[buf][1][wave] = sb;
    }
    store_row(ra, EA, sa, &sA[buf][0][wsw(am, ap)], &sA[buf][1][wsw(am, ap)]);
    store_row(rb, EB, sb, &sB[buf][0][wsw(bn, bp)], &sB[buf][1][wsw(bn, bp)]);
  };
  // staging wave of this lane's accumulator rows (per a, r) and columns (per b)
  auto wave_a = [&](int a, int r) { return (wm * (BM / 2) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) / RWA; };
  auto wave_b = [&](int b) { return (wn * (BN / 2) + b * 32 + li) / RWB; };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  f32x4 ua = {1.f, 1.f, 1.f, 1.f}, ub = {1.f, 1.f, 1.f, 1.f};  // accumulator units per staging wave
  const int nst = (p_end - p_begin + BK - 1) / BK;
  if (nst > 0) {
    gload(p_begin);
    lstore(0);
  }
  __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int cur = st & 1;
    if (st + 1 < nst) gload(p_begin + (st + 1) * BK);
    {  // this K-step's scales; re-express the partial sums in them (exact: powers of two)
      const f32x4 na = *reinterpret_cast<const f32x4*>(&sscale[cur][0][0]);
      const f32x4 nb = *reinterpret_cast<const f32x4*>(&sscale[cur][1][0]);
      if (st == 0) {
        ua = na;
        ub = nb;
      } else if (na[0] != ua[0] || na[1] != ua[1] || na[2] != ua[2] || na[3] != ua[3] || nb[0] != ub[0] ||
                 nb[1] != ub[1] || nb[2] != ub[2] || nb[3] != ub[3]) {
        float fa[4], fb[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          fa[q] = na[q] / ua[q];
          fb[q] = nb[q] / ub[q];
        }
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b) {
            const float f = fb[wave_b(b)];
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] *= fa[wave_a(a, r)] * f;
          }
        ua = na;
        ub = nb;
      }
    }
    f16x8 af[2][TM], bf[2][TN];
#pragma unroll
    for (int pl = 0; pl < 2; ++pl) {
#pragma unroll
      for (int a = 0; a < TM; ++a)
        af[pl][a] = *reinterpret_cast<const f16x8*>(&sA[cur][pl][wsw(wm * (BM / 2) + a * 32 + li, 8 * lh)]);
#pragma unroll
      for (int b = 0; b < TN; ++b)
        bf[pl][b] = *reinterpret_cast<const f16x8*>(&sB[cur][pl][wsw(wn * (BN / 2) + b * 32 + li, 8 * lh)]);
    }
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1][a], bf[0][b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0][a], bf[1][b], acc[a][b], 0, 0, 0);
        acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0][a], bf[0][b], acc[a][b], 0, 0, 0);
      }
    if (st + 1 < nst) lstore(cur ^ 1);
    __syncthreads();
  }
  float* out = g.part + (size_t)split * (g.split_stride ? g.split_stride : (int64_t)g.Mp * g.Np);
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int n = n0 + wn * (BN / 2) + b * 32 + li;
      const float ib = 1.f / ub[wave_b(b)];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * (BM / 2) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        out[(size_t)m * g.Np + n] = acc[a][b][r] * (ib / ua[wave_a(a, r)]);
      }
    }
  if (do_bias) {  // column sums of A: TPA partial sums per column (consecutive threads), fixed order
    float* red = reinterpret_cast<float*>(&sA[0][0][0]);
    red[tid] = bsum;
    __syncthreads();
    if (tid < BM) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < TPA; ++q) t += red[tid * TPA + q];
      g.part_bias[(size_t)split * g.Mp + m0 + tid] = t;
    }
  }
}

// The Winograd weight-gradient contraction in fp16x3 with the operands staged as they lie in
// memory (pis_tune key 31 = 1): a K-step is 32 pixel rows x 128 columns of A (E[t][Cout]) and of
// B (V[t][Cin]), loaded as float4s along the rows (512 contiguous bytes per 32 lanes), split into
// hi / lo fp16 planes [pixel][column] with ONE power-of-two scale per operand per K-step (the
// block-wide max, h3_keep), and the MFMA fragments (8 consecutive pixels of one column per lane)
// come out by transposed reads (ds_read_b64_tr_b16). Compared with wgrad_h3_kernel: 4x fewer
// global load instructions, twice the K per barrier, and the raw operands of K-step st + 2 in
// flight while K-step st multiplies (two register sets); the next K-step's split runs in this
// K-step's MFMA stream. Wave (wm, wn): rows 64 wm .., columns 64 wn .. of the 128 x 128 tile.
// LDS rows are 256 B; the 16-B chunk index is XORed with 4 (row & 3), so a transposed read's
// 32-lane half (4 rows x 4 chunks) meets 64 distinct banks and a row store (32 lanes) too.
constexpr int WT_BK = 32;                        // pixels per K-step
constexpr int WT_PLANE = WT_BK * 128;            // fp16 per plane
constexpr int WT_BUF = 4 * WT_PLANE;             // A hi, A lo, B hi, B lo

__device__ __forceinline__ int wtsw(int row, int chunk) { return row * 128 + 8 * (chunk ^ ((row & 3) << 2)); }

// UP2 (the transposed-conv weight gradient, pis_tune key 13 = 4): A(p, (i, j, o)) = dy at the
// up-sampled pixel (2y + i, 2x + j) of low-resolution pixel p = (b, y, x); with W % 32 == 0 and
// 32-aligned split starts a K-step's 32 pixels lie in one image row, so its rows are one base +
// 2 r pixels apart; the bias partials (column sums of A, blocks of the first column tile) are
// summed from the raw loads and reduced over the 8 threads of a column group in LDS (fixed order).
// TW: the timing-twin instantiation (pis_tune key 2 != 0 only; the production kernel has no debug branch)
// EX: every split is whole K-steps (P % 32 == 0; the plan's pps is a multiple of 32) and every
// operand row offset fits 31 bits: no per-row tail test, and the plain operands are read by
// buffer loads from the block's base (32-bit lane offset + a wave-uniform row offset per j)
// instead of 64-bit per-lane address arithmetic. Same loads, same sums (bitwise equal).
template <bool UP2 = false, int D = 2, bool TW = false, bool EX = false>
__global__ __launch_bounds__(256, 2) void wgrad_h3t_kernel(WgradArgs g) {
  const Remap2 rm = xcd_remap2();
  if (rm.batch) {
    g.a += rm.batch * g.bs_a;
    g.b += rm.batch * g.bs_b;
    g.part += rm.batch * g.bs_part;
  }
  __shared__ __attribute__((aligned(16))) _Float16 smem[2 * WT_BUF];
  __shared__ float red[2][2][4];  // [K-step parity][A|B][wave] maxima
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, lh = lane >> 5;
  const int ntn = g.Np / 128;
  const int tiles = (g.Mp / 128) * ntn;
  const int bid = rm.bid;
  const int split = bid / tiles;
  const int tile = bid - split * tiles;
  const int m0 = (tile / ntn) * 128, n0 = (tile % ntn) * 128;
  const int p_begin = split * g.pix_per_split;
  const int p_end = min(g.P, p_begin + g.pix_per_split);
  const int nst = max(0, (p_end - p_begin + WT_BK - 1) / WT_BK);
  // staging: item i = tid + 256 j -> pixel row i >> 5, float4 column (i & 31)
  const int srow = tid >> 5, sc4 = tid & 31;
  const float* ga = g.a + m0 + 4 * sc4;
  const float* gb = g.b + n0 + 4 * sc4;
  int up_ij = 0;
  if (UP2) {  // this thread's A column group: tap (i, j) = up_ij, channel o
    const int col = m0 + 4 * sc4;
    up_ij = col / g.Ca;
    ga = g.a + (col - up_ij * g.Ca);
  }
  // bias partials = column sums of A over the block's pixels: the transposed conv's dy (UP2), or the
  // Winograd weight gradient's E plane xi = bias_xi (E[7] = (1/3)^2 x the 4x4 tile's dz sum)
  const bool do_bias = g.part_bias != nullptr && n0 == 0 && rm.batch == g.bias_xi;
  f32x4 bsum = {0.f, 0.f, 0.f, 0.f};

  f32x4 ra[D][4], rb[D][4];
  // EX: buffer resources at the block's column bases; lane offsets of row p_begin + srow
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.a + m0), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(g.b + n0), (short)0, 0x7fffffff, 0x00020000);
  const uint32_t la0 = 4u * ((uint32_t)(p_begin + srow) * (uint32_t)g.lda + 4u * sc4);
  const uint32_t lb0 = 4u * ((uint32_t)(p_begin + srow) * (uint32_t)g.ldb + 4u * sc4);
  auto gload = [&](f32x4 (&xa)[4], f32x4 (&xb)[4], int st) __attribute__((always_inline)) {
    if (TW && (g.dbg & 1) && st >= D) return;
    if constexpr (EX) {  // rows p_begin + 32 st + srow + 8 j, all inside the split
      const uint32_t ra_s = 4u * (uint32_t)(st * WT_BK) * (uint32_t)g.lda, rb_s = 4u * (uint32_t)(st * WT_BK) * (uint32_t)g.ldb;
      size_t abase = 0;
      if (UP2) {
        const int p0 = p_begin + st * WT_BK;
        const int hw = g.H * g.W, b = p0 / hw, rem = p0 - b * hw, y = rem / g.W, x0 = rem - y * g.W;
        abase = (((size_t)b * 2 * g.H + 2 * y + (up_ij >> 1)) * (2 * g.W) + 2 * x0 + (up_ij & 1)) * g.lda;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (UP2)
          xa[j] = *reinterpret_cast<const f32x4*>(ga + abase + (size_t)(2 * (srow + 8 * j)) * g.lda);
        else
          xa[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsa, la0, ra_s + 4u * (uint32_t)(8 * j) * (uint32_t)g.lda, 0));
        xb[j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsb, lb0, rb_s + 4u * (uint32_t)(8 * j) * (uint32_t)g.ldb, 0));
      }
      return;
    }
    const int p0 = p_begin + st * WT_BK;
    size_t abase = 0;
    if (UP2) {  // the K-step's 32 pixels: one image row (b, y), columns x0 ..
      const int hw = g.H * g.W, pb = min(p0, p_end - 1);
      const int b = pb / hw, rem = pb - b * hw, y = rem / g.W, x0 = (rem - y * g.W) & ~31;
      abase = (((size_t)b * 2 * g.H + 2 * y + (up_ij >> 1)) * (2 * g.W) + 2 * x0 + (up_ij & 1)) * g.lda;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // rows past the split's end: a valid row loaded, zeros kept (no divergent branch)
      const int p = p0 + srow + 8 * j;
      const bool ok = p < p_end;
      const size_t pc = ok ? p : p_begin;
      const f32x4 va = UP2 ? *reinterpret_cast<const f32x4*>(ga + abase + (size_t)(ok ? 2 * (srow + 8 * j) : 0) * g.lda)
                           : *reinterpret_cast<const f32x4*>(ga + pc * g.lda);
      const f32x4 vb = *reinterpret_cast<const f32x4*>(gb + pc * g.ldb);
      xa[j] = ok ? va : f32x4{0.f, 0.f, 0.f, 0.f};
      xb[j] = ok ? vb : f32x4{0.f, 0.f, 0.f, 0.f};
    }
  };
  auto publish = [&](const f32x4 (&xa)[4], const f32x4 (&xb)[4], int par) __attribute__((always_inline)) {
    if (do_bias) {
#pragma unroll
      for (int j = 0; j < 4; ++j) bsum += xa[j];
    }
    const float ma = wave_max_nonneg(absmax_x4(xa));
    const float mb = wave_max_nonneg(absmax_x4(xb));
    if (lane == 0) {
      red[par][0][wave] = ma;
      red[par][1][wave] = mb;
    }
  };
  float sa_last = 0.f, sb_last = 0.f, sa_min = __builtin_inff(), sb_min = __builtin_inff();
  auto split_store = [&](const f32x4 (&xa)[4], const f32x4 (&xb)[4], int par, float& sa, float& sb) __attribute__((always_inline)) {
    auto umax4 = [](const float (&r)[4]) __attribute__((always_inline)) {  // r >= 0: bit-pattern max
      return __uint_as_float(max(max(__float_as_uint(r[0]), __float_as_uint(r[1])),
                                 max(__float_as_uint(r[2]), __float_as_uint(r[3]))));
    };
    const float ma = umax4(red[par][0]);
    const float mb = umax4(red[par][1]);
    sa = sa_last = h3_keep(sa_last, ma, sa_min);
    sb = sb_last = h3_keep(sb_last, mb, sb_min);
    _Float16* buf = smem + par * WT_BUF;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int off = wtsw(srow + 8 * j, sc4 >> 1) + 4 * (sc4 & 1);
      u32x2 h, l;
      split2h_x4(xa[j] * sa, h, l);
      *reinterpret_cast<u32x2*>(buf + off) = h;
      *reinterpret_cast<u32x2*>(buf + WT_PLANE + off) = l;
      split2h_x4(xb[j] * sb, h, l);
      *reinterpret_cast<u32x2*>(buf + 2 * WT_PLANE + off) = h;
      *reinterpret_cast<u32x2*>(buf + 3 * WT_PLANE + off) = l;
    }
  };

  // transposed-read lane roles: 16-lane group gq, its row q and 8-B slot p
  const int gq = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const int kh = gq >> 1, chk = 2 * (gq & 1) + (pp >> 1), slot = 4 * (pp & 1);
  auto frag = [&](const _Float16* plane, int ks, int col0) __attribute__((always_inline)) {
    const int row = 16 * ks + 8 * kh + q, ch = col0 / 8 + chk;
    const s16x4 lo4 = tr_read(plane + wtsw(row, ch) + slot);
    const s16x4 hi4 = tr_read(plane + wtsw(row + 4, ch) + slot);
    return __builtin_bit_cast(f16x8, __builtin_shufflevector(lo4, hi4, 0, 1, 2, 3, 4, 5, 6, 7));
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  // the partial sums are in units ua * ub, kept as TWO factors (0: none yet): each scale may be up
  // to 2^126 (common.h h2_scale_pair), so their product can overflow fp32 when both operands are
  // small (dz ~ 1e-30 against activations ~ 1e-2); the rescale and the epilogue apply one factor
  // at a time, every step an exact power of two
  float ua = 0.f, ub = 0.f;
  float s_a[2] = {0.f, 0.f}, s_b[2] = {0.f, 0.f};  // per buffer parity: the staged K-step's scales

  // D register sets: the raw operands of K-step st + D in flight while K-step st multiplies. Set
  // of K-step k: k % D; LDS buffer: k & 1. (D = 3 measured neutral on every C2 layer,
  // profiles/r3_q22_wgrad_depth.txt: D = 2 is launched.)
  if (nst > 0) {
#pragma unroll
    for (int k = 0; k < D; ++k)
      if (k < nst) gload(ra[k], rb[k], k);
    publish(ra[0], rb[0], 0);
    __syncthreads();
    split_store(ra[0], rb[0], 0, s_a[0], s_b[0]);
    if (nst > D) gload(ra[0], rb[0], D);
  }
  auto kstep = [&](int st, auto par_c, auto set_c) __attribute__((always_inline)) {
    constexpr int cur = decltype(par_c)::value, nxt = cur ^ 1;
    constexpr int sn = (decltype(set_c)::value + 1) % D;  // register set of K-step st + 1
    if (st + 1 < nst) publish(ra[sn], rb[sn], nxt);
    __syncthreads();  // buffer cur staged; buffer nxt's readers (K-step st - 1) done
    const _Float16* buf = smem + cur * WT_BUF;
    f16x8 af[2][2], bf[2][2];
#pragma unroll
    for (int pl = 0; pl < 2; ++pl)
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        af[pl][a] = frag(buf + pl * WT_PLANE, 0, 64 * wm + 32 * a);
        bf[pl][a] = frag(buf + (2 + pl) * WT_PLANE, 0, 64 * wn + 32 * a);
      }
    if (st + 1 < nst) {
      if (!(TW && (g.dbg & 2) && st > 0)) split_store(ra[sn], rb[sn], nxt, s_a[nxt], s_b[nxt]);
      if (st + 1 + D < nst) gload(ra[sn], rb[sn], st + 1 + D);
    }
    {  // the partial sums in this K-step's units (exact: powers of two, one factor at a time)
      const float sa = s_a[cur], sb = s_b[cur];
      if (sa != ua || sb != ub) {
        if (ua != 0.f) {
          const float fa = sa / ua, fb = sb / ub;
#pragma unroll
          for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b) acc[a][b] = (acc[a][b] * fa) * fb;
        }
        ua = sa;
        ub = sb;
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      if (ks) {
#pragma unroll
        for (int pl = 0; pl < 2; ++pl)
#pragma unroll
          for (int a = 0; a < 2; ++a) {
            af[pl][a] = frag(buf + pl * WT_PLANE, 1, 64 * wm + 32 * a);
            bf[pl][a] = frag(buf + (2 + pl) * WT_PLANE, 1, 64 * wn + 32 * a);
          }
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1][a], bf[0][b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0][a], bf[1][b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0][a], bf[0][b], acc[a][b], 0, 0, 0);
        }
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  if constexpr (D == 2) {
#pragma unroll 1
    for (int st = 0; st < nst; st += 2) {
      kstep(st, I0{}, I0{});
      if (st + 1 < nst) kstep(st + 1, I1{}, I1{});
    }
  } else {  // K-steps by six: buffer parity and register set both repeat
#pragma unroll 1
    for (int st = 0; st < nst; st += 6) {
      kstep(st, I0{}, I0{});
      if (st + 1 < nst) kstep(st + 1, I1{}, I1{});
      if (st + 2 < nst) kstep(st + 2, I0{}, I2{});
      if (st + 3 < nst) kstep(st + 3, I1{}, I0{});
      if (st + 4 < nst) kstep(st + 4, I0{}, I1{});
      if (st + 5 < nst) kstep(st + 5, I1{}, I2{});
    }
  }
  float* out = g.part + (size_t)split * (g.split_stride ? g.split_stride : (int64_t)g.Mp * g.Np);
  const float inv_a = ua != 0.f ? 1.f / ua : 0.f, inv_b = ub != 0.f ? 1.f / ub : 0.f;
  if (TW && (g.dbg & 4)) {
    float t = 0.f;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) t += acc[a][b][r];
    if (t == 1.2345f) out[tid] = t;
    return;
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int n = n0 + 64 * wn + 32 * b + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + 64 * wm + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * lh;
        out[(size_t)m * g.Np + n] = (acc[a][b][r] * inv_a) * inv_b;
      }
    }
  if (do_bias) {  // column sums over the block's pixels: the 8 threads of each column group
    __syncthreads();
    f32x4* rb4 = reinterpret_cast<f32x4*>(smem);
    rb4[tid] = bsum;
    __syncthreads();
    if (tid < 32) {
      f32x4 t = rb4[tid];
#pragma unroll
      for (int r = 1; r < 8; ++r) t += rb4[32 * r + tid];
      *reinterpret_cast<f32x4*>(g.part_bias + (size_t)split * g.Mp + m0 + 4 * tid) = t;
    }
  }
}

// wgrad_h3t_kernel's EX form: whole K-steps in every split (pix_per_split is a multiple of 32) and
// 31-bit row offsets for the buffer loads (the batch offsets go into the base pointers)
static bool h3t_exact(const WgradArgs& a) {
  return a.P % WT_BK == 0 && a.pix_per_split % WT_BK == 0 &&
         ((int64_t)a.P + WT_BK) * std::max(a.a_up2 ? 0 : a.lda, a.ldb) * 4 < (int64_t(1) << 31);
}

static int run_wgrad(const WgradArgs& base, const WgradPlan& pl, hipStream_t s, int batches = 1) {
  WgradArgs a = base;
  a.pix_per_split = pl.pps;
  a.pair = tune_get(PIS_TUNE_WGRAD_PAIR);
  a.dbg = tune_get(PIS_TUNE_DEBUG_NOLOAD);
  const int tiles = (a.Mp / pl.bm) * (a.Np / pl.bn);
  const dim3 grid(tiles * pl.splits, batches);
  // key 14 = 3 (auto): fp16x3 where the contraction's output has >= 256 columns (Cin): measured
  // per layer (profiles/r2_q53_wgrad_fp16x3.txt) it wins on exactly those (-1..-10 %) and loses on
  // the HBM-bound 64 / 128-channel layers (+1..+9 %). The split GEMMs take plain B operands only,
  // where Np IS the input-channel count (Winograd: Cin; convT: Cin); the direct path's B_CONV3
  // operand (Np = 9 Cin) never reaches them, it runs the fp32 MFMA kernel below
  const int x6 = tune_get(PIS_TUNE_WGRAD_X6);
  const bool plain = a.b_mode == B_PLAIN;
  const int cin = plain ? a.Np : a.Cb;
  if ((x6 == 2 || (x6 == 3 && cin >= 256)) && plain && pl.pps % 16 == 0 &&
      (!a.a_up2 || a.W % 8 == 0)) {
    // key 31: the row-staged kernel for plain 128 x 128 tiles (float4 rows: 16-B aligned)
    if (tune_get(PIS_TUNE_WGRAD_T) != 0 && pl.bm == 128 && pl.bn == 128 && !a.a_up2 &&
        pl.pps % WT_BK == 0 && a.lda % 4 == 0 && a.ldb % 4 == 0 && a.bs_a % 4 == 0 && a.bs_b % 4 == 0 &&
        ((uintptr_t)a.a & 15) == 0 && ((uintptr_t)a.b & 15) == 0) {
      if (a.dbg)
        hipLaunchKernelGGL((wgrad_h3t_kernel<false, 2, true>), grid, dim3(256), 0, s, a);
      else if (h3t_exact(a))
        hipLaunchKernelGGL((wgrad_h3t_kernel<false, 2, false, true>), grid, dim3(256), 0, s, a);
      else
        hipLaunchKernelGGL((wgrad_h3t_kernel<false, 2>), grid, dim3(256), 0, s, a);
      return launch_status("wgrad_h3t");
    }
    if (pl.bm == 128 && pl.bn == 128) hipLaunchKernelGGL((wgrad_h3_kernel<128, 128>), grid, dim3(256), 0, s, a);
    else if (pl.bm == 128) hipLaunchKernelGGL((wgrad_h3_kernel<128, 64>), grid, dim3(256), 0, s, a);
    else if (pl.bn == 128) hipLaunchKernelGGL((wgrad_h3_kernel<64, 128>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((wgrad_h3_kernel<64, 64>), grid, dim3(256), 0, s, a);
    return launch_status("wgrad_h3");
  }
  if (x6 != 0 && a.b_mode == B_PLAIN && pl.pps % 16 == 0 && (!a.a_up2 || a.W % 8 == 0)) {
    if (pl.bm == 128 && pl.bn == 128) hipLaunchKernelGGL((wgrad_x6_kernel<128, 128>), grid, dim3(256), 0, s, a);
    else if (pl.bm == 128) hipLaunchKernelGGL((wgrad_x6_kernel<128, 64>), grid, dim3(256), 0, s, a);
    else if (pl.bn == 128) hipLaunchKernelGGL((wgrad_x6_kernel<64, 128>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((wgrad_x6_kernel<64, 64>), grid, dim3(256), 0, s, a);
    return launch_status("wgrad_x6");
  }
  if (pl.bm == 128 && pl.bn == 128)
    hipLaunchKernelGGL((wgrad_f32_kernel<128, 128, 16>), grid, dim3(256), 0, s, a);
  else if (pl.bm == 128)
    hipLaunchKernelGGL((wgrad_f32_kernel<128, 64, 32>), grid, dim3(256), 0, s, a);
  else if (pl.bn == 128)
    hipLaunchKernelGGL((wgrad_f32_kernel<64, 128, 32>), grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((wgrad_f32_kernel<64, 64, 32>), grid, dim3(256), 0, s, a);
  return launch_status("wgrad_f32");
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

static WgradPlan conv_plan(int B, int H, int W, int Cin, int Cout) {
  const int P = B * H * W;
  if (Cin == 1) return plan_wgrad(Cout, 64, P, Cout, 64);
  return plan_wgrad(Cout, 9 * Cin, P, Cout, Cin);
}

struct HaloPlan {
  bool use;
  int splits, seg_per_split, nseg;
  size_t part_bytes, bias_bytes;
};

static HaloPlan halo_plan(int B, int H, int W, int Cin, int Cout) {
  HaloPlan p{};
  p.use = Cin % 64 == 0 && Cout % 64 == 0 && W % 16 == 0;
  if (!p.use) return p;
  p.nseg = (int)((int64_t)B * H * W / 16);
  const int tiles = (Cout / 64) * (Cin / 64);
  const size_t slab = (size_t)Cout * 9 * Cin * sizeof(float);
  // one round of blocks (2 per CU), 512..8192 pixels per split, <= ~160 MB of partial slabs
  int64_t splits = cdiv(std::max(64, tune_get(PIS_TUNE_WGRAD_BLOCKS)), tiles);
  splits = std::min<int64_t>(splits, std::max<int64_t>(1, (int64_t)((160u << 20) / slab)));
  int64_t sps = cdiv(p.nseg, splits);
  sps = std::max<int64_t>(32, std::min<int64_t>(512, sps));
  p.seg_per_split = (int)sps;
  p.splits = (int)cdiv(p.nseg, sps);
  p.part_bytes = (size_t)p.splits * slab;
  p.bias_bytes = (size_t)p.splits * Cout * sizeof(float);
  return p;
}

// Cin == 1 (enc1.conv0): dw[n][t] = sum_p dz[p][n] x[p + tap t], db[n] = sum_p dz[p][n].
// K = 9 is far too short for MFMA and the pass is a read of dz (4*Cout B/px): Cout/4 lanes
// per pixel hold 4 channels x (9 taps + bias) fp32 accumulators, the grid walks contiguous
// pixel ranges, per-block partials go through the deterministic slab reduction.
constexpr int C1_BLOCKS = 1024;

__global__ __launch_bounds__(256) void wgrad_c1_kernel(const float* __restrict__ x, int ldx,
                                                       const float* __restrict__ dz, int ldz, int B, int H,
                                                       int W, int Cout, int64_t pix_per_block,
                                                       float* __restrict__ part, float* __restrict__ part_b) {
  __shared__ f32x4 red[256][10];
  const int lanes = Cout / 4, groups = 256 / lanes;
  const int lp = threadIdx.x / lanes, q = threadIdx.x - lp * lanes, c4 = 4 * q;
  f32x4 acc[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int HW = H * W;
  const int64_t npix = (int64_t)B * HW;
  const int64_t p0 = (int64_t)blockIdx.x * pix_per_block, p1 = min(npix, p0 + pix_per_block);
  if (lp < groups) {
    for (int64_t p = p0 + lp; p < p1; p += groups) {
      const int b = (int)(p / HW), rem = (int)(p - (int64_t)b * HW), h = rem / W, wc = rem - h * W;
      const f32x4 dv = *reinterpret_cast<const f32x4*>(dz + p * ldz + c4);
      acc[9] += dv;
      const float* xb = x + (int64_t)b * HW * ldx;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int hh = h + t / 3 - 1, ww = wc + t % 3 - 1;
        const float xv = (hh >= 0 && hh < H && ww >= 0 && ww < W) ? xb[(int64_t)(hh * W + ww) * ldx] : 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[t][j] = fmaf(xv, dv[j], acc[t][j]);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 10; ++k) red[threadIdx.x][k] = acc[k];
  __syncthreads();
  // fixed-order sum over the pixel groups: output o = (n, k) with k = tap (0..8) or bias (9)
  for (int o = threadIdx.x; o < 10 * Cout; o += 256) {
    const int n = o / 10, k = o - n * 10, qq = n >> 2, j = n & 3;
    float sum = 0.f;
    for (int gi = 0; gi < groups; ++gi) sum += red[gi * lanes + qq][k][j];
    if (k < 9) part[(size_t)blockIdx.x * 9 * Cout + n * 9 + k] = sum;
    else if (part_b) part_b[(size_t)blockIdx.x * Cout + n] = sum;
  }
}

// Cin == 1, Cout == 64, W % 64 == 0: blocks walk segments of R image rows x 64 pixels
// (grid-stride, fixed grid so the partial slabs stay few); per segment the (R + 2) x 66 input
// window is staged in LDS and thread (pixel group t / 16, channel quad t % 16) accumulates pixels
// pg + 16 k of each row: dz is read with whole-pixel float4 rows (1 KB per wave instruction), no
// per-pixel index divisions; R = 4 (H % 4 == 0) puts 16 dz loads per thread between the barriers.
template <int R>
__global__ __launch_bounds__(256) void wgrad_c1_row_kernel(const float* __restrict__ x, int ldx,
                                                           const float* __restrict__ dz, int ldz, int B, int H,
                                                           int W, float* __restrict__ part,
                                                           float* __restrict__ part_b) {
  constexpr int Cout = 64, SEG = 64;
  __shared__ float xs[R + 2][SEG + 2];
  __shared__ f32x4 red[256][10];
  const int tid = threadIdx.x, c4 = (tid & 15) * 4, pg = tid >> 4;
  f32x4 acc[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int segs = W / SEG, hb = H / R;
  const int nseg = B * hb * segs;
  for (int sg = blockIdx.x; sg < nseg; sg += gridDim.x) {
    const int bh = sg / segs, w0 = (sg - bh * segs) * SEG;
    const int b = bh / hb, h0 = (bh - b * hb) * R;
    __syncthreads();  // the previous segment's window is no longer read
    for (int i = tid; i < (R + 2) * (SEG + 2); i += 256) {
      const int r = i / (SEG + 2), c = i - r * (SEG + 2);
      const int hh = h0 + r - 1, ww = w0 + c - 1;
      xs[r][c] = (hh >= 0 && hh < H && ww >= 0 && ww < W) ? x[(((size_t)b * H + hh) * W + ww) * ldx] : 0.f;
    }
    __syncthreads();
    const float* dzr = dz + (((size_t)b * H + h0) * W + w0) * ldz + c4;
    f32x4 dv[R][4];
#pragma unroll
    for (int rr = 0; rr < R; ++rr)
#pragma unroll
      for (int k = 0; k < 4; ++k) dv[rr][k] = *reinterpret_cast<const f32x4*>(dzr + ((size_t)rr * W + pg + 16 * k) * ldz);
#pragma unroll
    for (int rr = 0; rr < R; ++rr)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int px = pg + 16 * k;
        acc[9] += dv[rr][k];
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const float xv = xs[rr + t / 3][px + t % 3];
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[t][j] = fmaf(xv, dv[rr][k][j], acc[t][j]);
        }
      }
  }
#pragma unroll
  for (int k = 0; k < 10; ++k) red[tid][k] = acc[k];
  __syncthreads();
  // fixed-order sum over the 16 pixel groups: output o = (n, k), k = tap (0..8) or bias (9)
  for (int o = tid; o < 10 * Cout; o += 256) {
    const int n = o / 10, k = o - n * 10, qq = n >> 2, j = n & 3;
    float sum = 0.f;
    for (int gi = 0; gi < 16; ++gi) sum += red[gi * 16 + qq][k][j];
    if (k < 9) part[(size_t)blockIdx.x * 9 * Cout + n * 9 + k] = sum;
    else if (part_b) part_b[(size_t)blockIdx.x * Cout + n] = sum;
  }
}

// Winograd weight gradient (csrc/winograd.hip), F(3x3, 4x4) when the 4x4 tile grid fits (pis_tune
// key 11), else F(3x3, 2x2): V = B^T x B and E = G e G^T per tile, M_xi[n][c] = sum_tiles
// E_xi[t][n] V_xi[t][c] as nxi = (m+2)^2 batched split-K GEMMs over the T tiles (slabs
// [split][xi][Cout][Cin], one fixed-order reduction), dW = A^T M A; the bias gradient is a
// channel sum of dz.
struct WinoWgradPlan {
  bool use, fused_bias, gemm_bias;
  int m, nxi;
  int64_t T;
  WgradPlan gemm;
  size_t off_E, off_part, off_M, off_cs, total;
};

static WinoWgradPlan wino_wgrad_plan(int B, int H, int W, int Cin, int Cout) {
  WinoWgradPlan p{};
  const int mode = tune_get(PIS_TUNE_WINOGRAD);
  // auto (tools/bench_kernels.py --key 8 --variants 1,2 --ops wgrad, B=8): dec1.conv0 -25 %,
  // enc2.conv0 -15 %, 64 -> 64 -2 % against the halo kernel
  const int m = (tune_get(PIS_TUNE_WINO_F4) != 0 && H % 4 == 0 && W % 4 == 0) ? 4 : 2;
  // F(3x3,4x4) everywhere on 4-aligned grids (64 -> 64 at 512^2: -2 % alone, -27 % with the
  // forward's kept transform); F(3x3,2x2) only with >= 128 on both sides
  const bool wanted = m == 4 || (Cin >= 128 && Cout >= 128);
  p.use = mode != 0 && H % 2 == 0 && W % 2 == 0 && Cin % 64 == 0 && Cout % 64 == 0 && (mode == 2 || wanted);
  if (!p.use) return p;
  p.m = m;
  p.nxi = (p.m + 2) * (p.m + 2);
  p.T = (int64_t)B * (H / p.m) * (W / p.m);
  // the nxi GEMMs share one launch: split so all of them together make ~target blocks
  p.gemm = plan_wgrad(Cout, Cin, (int)p.T, Cout, Cin, std::max(16, tune_get(PIS_TUNE_WINO_WGRAD_BLOCKS) / p.nxi));
  auto al = [](size_t b) { return cdiv(b, 256) * 256; };
  const size_t V = al((size_t)p.nxi * p.T * Cin * 4), E = al((size_t)p.nxi * p.T * Cout * 4);
  const size_t part = al((size_t)p.gemm.splits * p.nxi * Cout * Cin * 4), M = al((size_t)p.nxi * Cout * Cin * 4);
  p.off_E = V;
  p.off_part = V + E;
  p.off_M = p.off_part + part;
  p.off_cs = p.off_M + M;
  // bias gradient. F(3x3,4x4): the GEMM's blocks of plane xi = 7 sum their E rows per column
  // (E[7] = (1/3)^2 x the tile's dz sum, w4_g4 row 1) into [split][Cout] partials, which the output
  // transform's bias blocks reduce in fixed order (no pass, no launch of its own). Else a
  // channel-sum pass over dz.
  p.gemm_bias = p.m == 4 && ((int64_t)Cout * Cin) % 64 == 0;
  p.fused_bias = false;
  const size_t cs = p.gemm_bias ? (size_t)p.gemm.splits * Cout * sizeof(float) : colsum_ws((int64_t)B * H * W, Cout);
  p.total = p.off_cs + al(cs) + 256;
  return p;
}

// bytes of the forward's F(4x4,3x3) input transform the weight gradient can take over
// (pis_conv3x3_keep_bytes): the same B^T on the same 6x6 patches
size_t wino_wgrad_keep_bytes(int B, int H, int W, int Cin, int Cout) {
  if (direct_w_wanted(B, H, W, Cin, Cout, 4, 4)) return 0;  // the direct weight gradient reads x itself
  if (wino6_layer(B, H, W, Cin, Cout)) return 0;  // an F(6x6) forward keeps no F(4x4) transform
  const WinoWgradPlan p = wino_wgrad_plan(B, H, W, Cin, Cout);
  return (p.use && p.m == 4) ? (size_t)p.nxi * p.T * Cin * sizeof(float) : 0;
}

static int wino_wgrad(const float* x, int ldx, const float* dz, int ldz, float* dw, float* db, int B, int H, int W,
                      int Cin, int Cout, int acc, const WinoWgradPlan& p, void* ws, hipStream_t s,
                      const float* keep_v = nullptr, bool e_ready = false) {
  char* base = (char*)ws;
  float* V = (float*)base;
  float* E = (float*)(base + p.off_E);
  float* part = (float*)(base + p.off_part);
  float* M = (float*)(base + p.off_M);
  int rc = 0;
  if (keep_v && p.m == 4) V = const_cast<float*>(keep_v);  // the forward's transform of x
  else rc = launch_wino_input(x, ldx, B, H, W, Cin, V, s, p.m);
  if (!rc && !e_ready) rc = launch_wino_dz(dz, ldz, B, H, W, Cout, E, s, p.m, nullptr);
  if (rc) return rc;
  float* gbias = (db && p.gemm_bias) ? (float*)(base + p.off_cs) : nullptr;
  WgradArgs a{};
  a.a = E; a.lda = Cout; a.a_up2 = 0; a.Ca = Cout;
  a.b = V; a.ldb = Cin; a.b_mode = B_PLAIN; a.Cb = Cin;
  a.B = 1; a.H = 1; a.W = (int)p.T; a.P = (int)p.T; a.Mp = Cout; a.Np = Cin;
  a.part = part; a.part_bias = gbias; a.bias_xi = WINO4_BIAS_XI;
  a.bs_a = p.T * Cout; a.bs_b = p.T * Cin; a.bs_part = (int64_t)Cout * Cin;
  a.split_stride = (int64_t)p.nxi * Cout * Cin;
  const double flop = 2.0 * p.nxi * (double)p.T * Cout * Cin;
  launch_hook("wino_wgrad_gemm", 0, s, flop);
  rc = run_wgrad(a, p.gemm, s, p.nxi);
  launch_hook("wino_wgrad_gemm", 1, s, flop);
  // up to 16 split slabs: the output transform sums them itself (no reduced copy of the 36 planes:
  // the separate slab reduction of a 14-slab 128 x 256 layer read 66 MB at 0.8 TB/s); many slabs
  // keep the parallel slab reduction
  const WgradOutBias bf{gbias, gbias ? p.gemm.splits : 0, db, WINO4_BIAS_SCALE};
  if (p.m == 4 && p.gemm.splits <= 16) {
    if (!rc) rc = launch_wino_wgrad_out(part, Cout, Cin, dw, acc, s, p.m, p.gemm.splits, a.split_stride, bf);
  } else {
    if (!rc) rc = reduce_slabs_pitched(part, p.gemm.splits, a.split_stride, a.split_stride, M, 0, s);
    if (!rc) rc = launch_wino_wgrad_out(M, Cout, Cin, dw, acc, s, p.m, 1, 0, bf);
  }
  if (!rc && db && !gbias) rc = colsum(dz, ldz, (int64_t)B * H * W, Cout, db, acc, base + p.off_cs, p.total - p.off_cs, s);
  return rc;
}

// workspace of the non-direct weight-gradient paths (Winograd, halo, generic)
static size_t wgrad_ws_nodirect(int B, int H, int W, int Cin, int Cout) {
  const WinoWgradPlan wp = wino_wgrad_plan(B, H, W, Cin, Cout);
  if (wp.use) return wp.total;
  const HaloPlan hp = halo_plan(B, H, W, Cin, Cout);
  if (hp.use) return cdiv(hp.part_bytes, 256) * 256 + hp.bias_bytes + 256;
  if (Cin == 1 && tune_get(PIS_TUNE_C1_WGRAD) == 0)
    return (size_t)C1_BLOCKS * 10 * Cout * sizeof(float) + 512;
  const WgradPlan pl = conv_plan(B, H, W, Cin, Cout);
  // Cin == 1 computes a padded [Cout][64] tile and compacts it through a staging slab
  const size_t stage = Cin == 1 ? (size_t)Cout * 64 * sizeof(float) + 256 : 0;
  return wgrad_ws_bytes(pl) + stage;
}

extern "C" size_t pis_conv3x3_wgrad_ws(int B, int H, int W, int Cin, int Cout) {
  if (direct_w_wanted(B, H, W, Cin, Cout, 4, 4)) return direct_w_ws_bytes(B, H, W, Cin, Cout);
  return wgrad_ws_nodirect(B, H, W, Cin, Cout);
}

__global__ void compact_c1_kernel(const float* __restrict__ full, float* __restrict__ dw, int Cout,
                                  int accumulate) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Cout * 9) return;
  const int n = i / 9, t = i - n * 9;
  const float v = full[n * 64 + t];
  dw[i] = accumulate ? dw[i] + v : v;
}

extern "C" int pis_conv3x3_wgrad_keep(const float* x, int ldx, const float* dz, int ldz, float* dw_krsc,
                                      float* db, int B, int H, int W, int Cin, int Cout, int flags, void* ws,
                                      size_t ws_bytes, const float* keep, pis_stream_t stream) {
  const WinoWgradPlan wp = wino_wgrad_plan(B, H, W, Cin, Cout);
  const bool prepared = flags & PIS_WINO_PREPARED;
  PIS_CHECK_ARG(!prepared || (keep && wp.use && wp.m == 4),
                "pis_conv3x3_wgrad_keep: PIS_WINO_PREPARED needs the kept-transform F(3x3,4x4) path");
  if (!keep || !(wp.use && wp.m == 4) || (!prepared && direct_w_wanted(B, H, W, Cin, Cout, ldx, ldz)))
    return pis_conv3x3_wgrad(x, ldx, dz, ldz, dw_krsc, db, B, H, W, Cin, Cout, flags, ws, ws_bytes, stream);
  PIS_CHECK_ARG(x && dz && dw_krsc && ldz % 4 == 0, "pis_conv3x3_wgrad_keep: bad arguments");
  PIS_CHECK_ARG(ws && ws_bytes >= wp.total, "pis_conv3x3_wgrad_keep: workspace too small");
  return wino_wgrad(x, ldx, dz, ldz, dw_krsc, db, B, H, W, Cin, Cout, flags & PIS_ACCUMULATE, wp, ws,
                    (hipStream_t)stream, keep, prepared);
}

extern "C" int pis_conv3x3_bwd_prep(const float* dz, int ldz, int B, int H, int W, int Cin, int Cout,
                                    void* ws_dgrad, size_t ws_dgrad_bytes, void* ws_wgrad, size_t ws_wgrad_bytes,
                                    pis_stream_t stream) {
  PIS_CHECK_ARG(dz && B > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0, "pis_conv3x3_bwd_prep: bad arguments");
  if (direct_w_wanted(B, H, W, Cin, Cout, 4, ldz)) return 0;  // direct kernels read dz themselves
  const WinoWgradPlan wp = wino_wgrad_plan(B, H, W, Cin, Cout);
  if (tune_get(PIS_TUNE_WINO_DZ2) == 0 || !ws_dgrad || !ws_wgrad || !(wp.use && wp.m == 4) ||
      Cin % 64 || Cout % 64 ||  // pis_conv3x3_wgrad_keep's channel contract
      ws_wgrad_bytes < wp.total || ldz % 4 || !dgrad_wino4_planned(B, H, W, Cin, Cout, ldz, ws_dgrad_bytes))
    return 0;  // not applicable: the two calls transform dz themselves
  float* V = wino_v_slot(ws_dgrad, Cout, Cin);
  char* base = (char*)ws_wgrad;
  float* E = (float*)(base + wp.off_E);
  float* tmax = wino_fused_h3_planned(B, H, W, Cout, Cin) ? wino_tmax_slot(ws_dgrad, B, H, W, Cout, Cin) : nullptr;
  // (no bias partials: the weight gradient's GEMM sums them from E, wino_wgrad_plan gemm_bias)
  const int rc = launch_wino_dz2(dz, ldz, B, H, W, Cout, V, E, nullptr, (hipStream_t)stream, tmax);
  // the dgrad_ex that consumes this V checks that it decides the same tile-maxima format
  if (!rc) wino_prep_record(ws_dgrad, B, H, W, Cout, Cin, tmax != nullptr);
  return rc ? rc : 1;
}

extern "C" int pis_conv3x3_wgrad(const float* x, int ldx, const float* dz, int ldz, float* dw_krsc,
                                 float* db, int B, int H, int W, int Cin, int Cout, int flags,
                                 void* ws, size_t ws_bytes, pis_stream_t stream) {
  PIS_CHECK_ARG(x && dz && dw_krsc && B > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0,
                "pis_conv3x3_wgrad: bad arguments");
  PIS_CHECK_ARG(ws && ws_bytes >= pis_conv3x3_wgrad_ws(B, H, W, Cin, Cout),
                "pis_conv3x3_wgrad: workspace too small");
  PIS_CHECK_ARG(Cout % 64 == 0 && (Cin == 1 || Cin % 64 == 0),
                "pis_conv3x3_wgrad: Cout must be a multiple of 64 and Cin 1 or a multiple of 64");
  PIS_CHECK_ARG((Cin == 1 || ldx % 4 == 0) && ldz % 4 == 0, "pis_conv3x3_wgrad: ld must be multiples of 4");
  hipStream_t s = (hipStream_t)stream;
  const int acc = flags & PIS_ACCUMULATE;
  // the direct kernel reads x and dz as float4s: 16-B aligned base pointers (a channel slice at an
  // offset that is not a multiple of 4 floats falls through to the Winograd / halo kernels)
  if (direct_w_wanted(B, H, W, Cin, Cout, ldx, ldz)) {
    // (a workspace smaller than the direct kernel's slabs falls through to the kernels below, as
    // does a misaligned operand)
    if (((uintptr_t)x & 15) == 0 && ((uintptr_t)dz & 15) == 0 && ws_bytes >= direct_w_ws_bytes(B, H, W, Cin, Cout))
      return launch_direct_wgrad(x, ldx, dz, ldz, dw_krsc, db, B, H, W, Cin, Cout, acc, ws, ws_bytes, s);
    PIS_CHECK_ARG(ws_bytes >= wgrad_ws_nodirect(B, H, W, Cin, Cout),
                  "pis_conv3x3_wgrad: x / dz not 16-byte aligned or workspace below the direct kernel's; "
                  "the non-direct fallback needs a larger "
                  "workspace than pis_conv3x3_wgrad_ws reports for this (direct) layer");
  }
  const WinoWgradPlan wp = wino_wgrad_plan(B, H, W, Cin, Cout);
  if (wp.use && ldx % 4 == 0 && ws_bytes >= wp.total)
    return wino_wgrad(x, ldx, dz, ldz, dw_krsc, db, B, H, W, Cin, Cout, acc, wp, ws, s);
  const HaloPlan hp = halo_plan(B, H, W, Cin, Cout);
  if (hp.use && ldx % 4 == 0) {
    W3Args a{};
    a.x = x; a.ldx = ldx; a.dz = dz; a.ldz = ldz;
    a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout;
    a.seg_per_split = hp.seg_per_split; a.nseg = hp.nseg;
    a.part = (float*)ws;
    a.part_bias = db ? (float*)((char*)ws + cdiv(hp.part_bytes, 256) * 256) : nullptr;
    const int tiles = (Cout / 64) * (Cin / 64);
    const double flop = 2.0 * (double)B * H * W * Cout * 9.0 * Cin;
    launch_hook("wgrad3x3_halo", 0, s, flop);
    if (tune_get(PIS_TUNE_WGRAD_VARIANT) != 0)
      hipLaunchKernelGGL((wgrad3x3_halo_kernel<2>), dim3(tiles * hp.splits), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((wgrad3x3_halo_kernel<1>), dim3(tiles * hp.splits), dim3(256), 0, s, a);
    launch_hook("wgrad3x3_halo", 1, s, flop);
    int rc = launch_status("wgrad3x3_halo");
    if (!rc) rc = reduce_slabs2(a.part, hp.splits, (int64_t)Cout * 9 * Cin, dw_krsc, a.part_bias, hp.splits, Cout, db,
                                acc, s);
    return rc;
  }
  if (Cin == 1 && tune_get(PIS_TUNE_C1_WGRAD) == 0) {
    PIS_CHECK_ARG(Cout <= 1024 && Cout % 4 == 0, "pis_conv3x3_wgrad: Cin == 1 needs Cout % 4 == 0, <= 1024");
    const int64_t npix = (int64_t)B * H * W;
    const int64_t ppb = cdiv(npix, C1_BLOCKS);
    const int blocks = (int)cdiv(npix, ppb);
    float* part = (float*)ws;
    float* part_b = db ? part + (size_t)C1_BLOCKS * 9 * Cout : nullptr;
    const bool row = Cout == 64 && W % 64 == 0 && ldz % 4 == 0;
    if (row && H % 4 == 0)
      hipLaunchKernelGGL(wgrad_c1_row_kernel<4>, dim3(C1_BLOCKS), dim3(256), 0, s, x, ldx, dz, ldz, B, H, W, part,
                         part_b);
    else if (row)
      hipLaunchKernelGGL(wgrad_c1_row_kernel<1>, dim3(C1_BLOCKS), dim3(256), 0, s, x, ldx, dz, ldz, B, H, W, part,
                         part_b);
    else
      hipLaunchKernelGGL(wgrad_c1_kernel, dim3(blocks), dim3(256), 0, s, x, ldx, dz, ldz, B, H, W, Cout, ppb,
                         part, part_b);
    int rc = launch_status("wgrad_c1");
    const int nslab = row ? C1_BLOCKS : blocks;
    if (!rc) rc = reduce_slabs2(part, nslab, (int64_t)9 * Cout, dw_krsc, db ? part_b : nullptr, nslab, Cout, db, acc, s);
    return rc;
  }
  const WgradPlan pl = conv_plan(B, H, W, Cin, Cout);
  WgradArgs a{};
  a.a = dz; a.lda = ldz; a.a_up2 = 0; a.Ca = Cout;
  a.b = x; a.ldb = ldx; a.b_mode = Cin == 1 ? B_CONV3_C1 : B_CONV3; a.Cb = Cin;
  a.B = B; a.H = H; a.W = W; a.P = B * H * W; a.Mp = Cout; a.Np = Cin == 1 ? 64 : 9 * Cin;
  a.part = (float*)ws;
  a.part_bias = db ? bias_slabs(ws, pl) : nullptr;
  int rc = run_wgrad(a, pl, s);
  if (rc) return rc;
  if (Cin == 1) {
    float* full = (float*)((char*)ws + wgrad_ws_bytes(pl));
    rc = reduce_slabs(a.part, pl.splits, (int64_t)Cout * 64, full, 0, s);
    if (!rc) {
      hipLaunchKernelGGL(compact_c1_kernel, dim3((unsigned)cdiv(Cout * 9, 256)), dim3(256), 0, s, full,
                         dw_krsc, Cout, acc);
      rc = launch_status("compact_c1");
    }
  } else {
    return reduce_slabs2(a.part, pl.splits, (int64_t)a.Mp * a.Np, dw_krsc, a.part_bias, pl.splits, Cout, db, acc, s);
  }
  if (rc || !db) return rc;
  return reduce_slabs(a.part_bias, pl.splits, Cout, db, acc, s);
}

// key 13 = 4: the transposed-conv weight gradient on the row-staged fp16x3 kernel (wgrad_h3t<UP2>)
// where it has >= 256 input channels (up2 -11 %, up3 -12 %, up4 -25 %; up1, 128 -> 64 at 256^2,
// +17 %: it keeps the bf16x6 column-staged kernel; profiles/r3_q17_convt.txt)
static bool convt_wgrad_t_ok(int B, int H, int W, int Cin, int Cout, int ldx, int lddy, const void* x,
                             const void* dy) {
  return tune_get(PIS_TUNE_CONVT_GEMM) == 4 && W % 32 == 0 && (4 * Cout) % 128 == 0 && Cin >= 256 && Cin % 128 == 0 &&
         ldx % 4 == 0 && lddy % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)dy & 15) == 0 &&
         plan_wgrad(4 * Cout, Cin, B * H * W, 4 * Cout, Cin).pps % WT_BK == 0;
}

extern "C" size_t pis_convt2x2_wgrad_ws(int B, int H, int W, int Cin, int Cout) {
  // either plan (key 13 may change after the workspace is sized)
  return std::max(wgrad_ws_bytes(plan_wgrad(4 * Cout, Cin, B * H * W, Cout, Cin)),
                  wgrad_ws_bytes(plan_wgrad(4 * Cout, Cin, B * H * W, 4 * Cout, Cin)));
}

extern "C" int pis_convt2x2_wgrad(const float* x, int ldx, const float* dy, int lddy, float* dw_ijoc,
                                  float* db, int B, int H, int W, int Cin, int Cout, int flags,
                                  void* ws, size_t ws_bytes, pis_stream_t stream) {
  PIS_CHECK_ARG(x && dy && dw_ijoc && B > 0 && H > 0 && W > 0 && Cin > 0 && Cout > 0,
                "pis_convt2x2_wgrad: bad arguments");
  PIS_CHECK_ARG(Cin % 64 == 0 && Cout % 64 == 0, "pis_convt2x2_wgrad: Cin/Cout must be multiples of 64");
  PIS_CHECK_ARG(ldx % 4 == 0 && lddy % 4 == 0, "pis_convt2x2_wgrad: ld must be multiples of 4");
  PIS_CHECK_ARG(ws && ws_bytes >= pis_convt2x2_wgrad_ws(B, H, W, Cin, Cout),
                "pis_convt2x2_wgrad: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const int acc = flags & PIS_ACCUMULATE;
  const int P = B * H * W;
  if (convt_wgrad_t_ok(B, H, W, Cin, Cout, ldx, lddy, x, dy)) {
    const WgradPlan pl = plan_wgrad(4 * Cout, Cin, P, 4 * Cout, Cin);  // 128 x 128 tiles (taps may share one)
    WgradArgs a{};
    a.a = dy; a.lda = lddy; a.a_up2 = 1; a.Ca = Cout;
    a.b = x; a.ldb = ldx; a.b_mode = B_PLAIN; a.Cb = Cin;
    a.B = B; a.H = H; a.W = W; a.P = P; a.Mp = 4 * Cout; a.Np = Cin; a.part = (float*)ws;
    a.part_bias = db ? bias_slabs(ws, pl) : nullptr;
    a.pix_per_split = pl.pps;
    const int tiles = (a.Mp / 128) * (a.Np / 128);
    if (h3t_exact(a))
      hipLaunchKernelGGL((wgrad_h3t_kernel<true, 2, false, true>), dim3(tiles * pl.splits), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((wgrad_h3t_kernel<true, 2>), dim3(tiles * pl.splits), dim3(256), 0, s, a);
    int rc = launch_status("wgrad_h3t<up2>");
    // weights + bias (slabs [split][i][j][o]: 4 splits slabs of Cout) in one launch
    if (!rc) rc = reduce_slabs2(a.part, pl.splits, (int64_t)a.Mp * a.Np, dw_ijoc, a.part_bias, pl.splits * 4, Cout, db,
                                acc, s);
    return rc;
  }
  const WgradPlan pl = plan_wgrad(4 * Cout, Cin, P, Cout, Cin);
  WgradArgs a{};
  a.a = dy; a.lda = lddy; a.a_up2 = 1; a.Ca = Cout;
  a.b = x; a.ldb = ldx; a.b_mode = B_PLAIN; a.Cb = Cin;
  a.B = B; a.H = H; a.W = W; a.P = P; a.Mp = 4 * Cout; a.Np = Cin; a.part = (float*)ws;
  a.part_bias = db ? bias_slabs(ws, pl) : nullptr;
  int rc = run_wgrad(a, pl, s);
  // weights + bias (slabs [split][i][j][o]: 4 splits slabs of Cout) in one launch
  if (!rc) rc = reduce_slabs2(a.part, pl.splits, (int64_t)a.Mp * a.Np, dw_ijoc, a.part_bias, pl.splits * 4, Cout, db,
                              acc, s);
  return rc;
}
