// ConvTranspose2d(k=2, s=2) of the U-Net decoder (src/unet.py:132-153) as lean NT GEMMs on
// fp32 MFMA (the Winograd GEMM's pipeline, csrc/winograd.hip:gemm_nt_kernel) with the
// transposed conv's addressing folded into the operand loads and the epilogue:
//
//   forward  y[b, 2i+di, 2j+dj, o] = bias[o] + sum_c x[b,i,j,c] w[di][dj][o][c]
//            GEMM M = B*h*w input pixels, N = 4*Cout (n = (2 di + dj) Cout + o), K = Cin;
//            A = x rows (ldx), Bt = w_ijoc rows; the epilogue scatters each 2x2 pixel block
//            into the concat slice (ldy) and adds the bias.
//   dgrad    dx[b,i,j,c] = [x > 0] sum_{di,dj,o} dy[b, 2i+di, 2j+dj, o] w[di][dj][o][c]
//            GEMM M = B*h*w, N = Cin, K = 4*Cout (k = (2 di + dj) Cout + o); A gathers the 2x2
//            output-gradient block (a 16-wide K chunk never straddles a tap when Cout % 16 == 0),
//            Bt = w_cijo rows (pis_convt2x2_prep); the epilogue applies the ReLU mask of the
//            convT input and optionally accumulates.
// Block tile 128 x 128, 4 waves of 64 x 64 (2 x 2 32x32 MFMA tiles), K-step 16 through a
// register-staged LDS double buffer; XCD-aware tile order. pis_tune key 13: 3 (default) fp16x3 on
// fp16 MFMA (fp32-class, -3..-18 % per layer vs bf16x6, profiles/r2_q68_*), 1 bf16x6 on bf16 MFMA
// (fp32-accurate), 2 native fp32 MFMA, 0 off (implicit-GEMM fallback).
#include "igemm.h"

namespace pis {

struct ConvtGemmArgs {
  const float* a;   // x (fwd) or dy (dgrad)
  int lda;          // channel stride of a
  const float* bt;  // w_ijoc [4 Cout][Cin] (fwd) or w_cijo [Cin][4 Cout] (dgrad)
  int B, h, w;      // input-pixel grid (the GEMM rows)
  int cin, cout;
  int M, N, K;
  // epilogue
  const float* bias;  // fwd
  const float* mask;  // dgrad (PIS_MASK)
  int ldm;
  float* dst;
  int ldd;
  int flags;
};

typedef __bf16 cbf16x8 __attribute__((ext_vector_type(8)));

// AR (arithmetic): 0 native fp32 MFMA; 1 X6: the operands are split into hi/mid/lo bf16 planes at
// LDS staging and every fp32 multiply-add becomes six bf16 MFMA partial products (fp32 accuracy,
// see gemm_nt_x6_kernel); 2 H3: fp16x3 (common.h) — hi/lo fp16 planes of the operands scaled by a
// power of two per wave and K-step (h3_keep), three fp16 products, accumulators re-expressed when
// a K-step's scales change (as wgrad_h3_kernel). Row r of a 128-row tile is staged by wave
// (r / 16) % 4 (threads tid / 4 and 64 + tid / 4).
template <int MODE, int AR>  // MODE 0 forward, 1 input gradient
__global__ __launch_bounds__(256, 2) void convt_gemm_kernel(ConvtGemmArgs g) {
  constexpr bool X6 = AR == 1, H3 = AR == 2;
  constexpr int BM = 128, BN = 128, BK = 16, ROW = BK + 4;
  constexpr int AL = BM * 4 / 256, BL = BN * 4 / 256;
  // LDS image per buffer: fp32 [row][ROW], or (X6) bf16 [hi|mid|lo][row][16] in the same floats
  constexpr int SA = X6 ? 3 * BM * BK / 2 : BM * ROW, SB = X6 ? 3 * BN * BK / 2 : BN * ROW;
  __shared__ __attribute__((aligned(16))) float sA[2][SA];
  __shared__ __attribute__((aligned(16))) float sB[2][SB];
  __shared__ __attribute__((aligned(16))) float sscale[2][2][4];  // H3: [buf][A|B][staging wave]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, lh = lane >> 5;
  const int ntn = (g.N + BN - 1) / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid / ntn) * BM, n0 = (bid % ntn) * BN;
  const int q4 = (tid & 3) * 4;
  const int hw = g.h * g.w;

  // per staged A row: the source pixel (fwd: the input pixel; dgrad: the top-left of its
  // 2x2 block in the 2h x 2w output-gradient grid)
  int64_t arow[AL];
  bool aok[AL];
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int m = m0 + (tid + i * 256) / 4;
    aok[i] = m < g.M;
    const int mm = aok[i] ? m : 0;
    if (MODE == 0) {
      arow[i] = mm;
    } else {
      const int b = mm / hw, rem = mm - b * hw, y = rem / g.w, x = rem - y * g.w;
      arow[i] = ((int64_t)b * 2 * g.h + 2 * y) * (2 * g.w) + 2 * x;
    }
  }
  f32x4 ra[AL], rb[BL];
  auto gload = [&](int k0) {
    int64_t tap = 0;
    int c = k0 + q4;
    if (MODE == 1) {  // k = (2 di + dj) Cout + o; the 16-wide chunk stays inside one tap
      const int ij = k0 / g.cout;
      c = k0 - ij * g.cout + q4;
      tap = (int64_t)(ij >> 1) * (2 * g.w) + (ij & 1);
    }
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (aok[i]) ra[i] = *reinterpret_cast<const f32x4*>(g.a + (arow[i] + tap) * g.lda + c);
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int n = n0 + (tid + i * 256) / 4;
      rb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (n < g.N) rb[i] = *reinterpret_cast<const f32x4*>(g.bt + (size_t)n * g.K + k0 + q4);
    }
  };
  float sa = 0.f, sb = 0.f;  // H3: this wave's current scales
  float sa_min = __builtin_inff(), sb_min = __builtin_inff();  // ... and the smallest so far
  auto lstore = [&](int buf) {
    if constexpr (H3) {
      sa = h3_keep(sa, wave_max_nonneg(absmax_x4(ra)), sa_min);
      sb = h3_keep(sb, wave_max_nonneg(absmax_x4(rb)), sb_min);
      if (lane == 0) {
        sscale[buf][0][wave] = sa;
        sscale[buf][1][wave] = sb;
      }
      _Float16* pa = reinterpret_cast<_Float16*>(sA[buf]);
      _Float16* pb = reinterpret_cast<_Float16*>(sB[buf]);
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        u32x2 h, l;
        split2h_x4(ra[i] * sa, h, l);
        const int o = wsw((tid + i * 256) / 4, q4);
        *reinterpret_cast<u32x2*>(pa + o) = h;
        *reinterpret_cast<u32x2*>(pa + BM * BK + o) = l;
      }
#pragma unroll
      for (int i = 0; i < BL; ++i) {
        u32x2 h, l;
        split2h_x4(rb[i] * sb, h, l);
        const int o = wsw((tid + i * 256) / 4, q4);
        *reinterpret_cast<u32x2*>(pb + o) = h;
        *reinterpret_cast<u32x2*>(pb + BN * BK + o) = l;
      }
    } else if constexpr (X6) {
      __bf16* pa = reinterpret_cast<__bf16*>(sA[buf]);
      __bf16* pb = reinterpret_cast<__bf16*>(sB[buf]);
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        u32x2 h, m, l;
        split3_x4(ra[i], h, m, l);
        const int o = wsw((tid + i * 256) / 4, q4);  // swizzled rows: conflict-free fragment reads
        *reinterpret_cast<u32x2*>(pa + o) = h;
        *reinterpret_cast<u32x2*>(pa + BM * BK + o) = m;
        *reinterpret_cast<u32x2*>(pa + 2 * BM * BK + o) = l;
      }
#pragma unroll
      for (int i = 0; i < BL; ++i) {
        u32x2 h, m, l;
        split3_x4(rb[i], h, m, l);
        const int o = wsw((tid + i * 256) / 4, q4);
        *reinterpret_cast<u32x2*>(pb + o) = h;
        *reinterpret_cast<u32x2*>(pb + BN * BK + o) = m;
        *reinterpret_cast<u32x2*>(pb + 2 * BN * BK + o) = l;
      }
    } else {
#pragma unroll
      for (int i = 0; i < AL; ++i) *reinterpret_cast<f32x4*>(&sA[buf][((tid + i * 256) / 4) * ROW + q4]) = ra[i];
#pragma unroll
      for (int i = 0; i < BL; ++i) *reinterpret_cast<f32x4*>(&sB[buf][((tid + i * 256) / 4) * ROW + q4]) = rb[i];
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  // H3: staging wave of this lane's accumulator rows (per a, r) and columns (per b); the
  // accumulators' units per staging wave
  auto wave_a = [&](int a, int r) { return ((wm * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) >> 4) & 3; };
  auto wave_b = [&](int b) { return ((wn * 64 + b * 32 + li) >> 4) & 3; };
  f32x4 ua = {1.f, 1.f, 1.f, 1.f}, ub = {1.f, 1.f, 1.f, 1.f};
  const int KT = g.K / BK;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) gload((kt + 1) * BK);
    if constexpr (H3) {
      // this K-step's scales; re-express the partial sums in them (exact: powers of two)
      const f32x4 na = *reinterpret_cast<const f32x4*>(&sscale[cur][0][0]);
      const f32x4 nb = *reinterpret_cast<const f32x4*>(&sscale[cur][1][0]);
      if (kt == 0) {
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
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const float f = fb[wave_b(b)];
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] *= fa[wave_a(a, r)] * f;
          }
        ua = na;
        ub = nb;
      }
      const _Float16* pa = reinterpret_cast<const _Float16*>(sA[cur]);
      const _Float16* pb = reinterpret_cast<const _Float16*>(sB[cur]);
      f16x8 af[2][2], bf[2][2];  // lane: row li, k = 8 lh .. 8 lh + 7
#pragma unroll
      for (int p = 0; p < 2; ++p) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
          af[p][a] = *reinterpret_cast<const f16x8*>(pa + p * BM * BK + wsw(wm * 64 + a * 32 + li, 8 * lh));
#pragma unroll
        for (int b = 0; b < 2; ++b)
          bf[p][b] = *reinterpret_cast<const f16x8*>(pb + p * BN * BK + wsw(wn * 64 + b * 32 + li, 8 * lh));
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {  // smallest partial products first
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1][a], bf[0][b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0][a], bf[1][b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0][a], bf[0][b], acc[a][b], 0, 0, 0);
        }
    } else if constexpr (X6) {
      const __bf16* pa = reinterpret_cast<const __bf16*>(sA[cur]);
      const __bf16* pb = reinterpret_cast<const __bf16*>(sB[cur]);
      cbf16x8 af[3][2], bf[3][2];  // lane: row li, k = 8 lh .. 8 lh + 7
#pragma unroll
      for (int p = 0; p < 3; ++p) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
          af[p][a] = *reinterpret_cast<const cbf16x8*>(pa + p * BM * BK + wsw(wm * 64 + a * 32 + li, 8 * lh));
#pragma unroll
        for (int b = 0; b < 2; ++b)
          bf[p][b] = *reinterpret_cast<const cbf16x8*>(pb + p * BN * BK + wsw(wn * 64 + b * 32 + li, 8 * lh));
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {  // smallest partial products first
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[2][a], bf[0][b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][a], bf[1][b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][a], bf[2][b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[1][a], bf[0][b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][a], bf[1][b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[0][a], bf[0][b], acc[a][b], 0, 0, 0);
        }
    } else {
#pragma unroll
    for (int gg = 0; gg < BK / 8; ++gg) {
      f32x4 af[2], bf[2];
#pragma unroll
      for (int a = 0; a < 2; ++a)
        af[a] = *reinterpret_cast<const f32x4*>(&sA[cur][(wm * 64 + a * 32 + li) * ROW + 8 * gg + 4 * lh]);
#pragma unroll
      for (int b = 0; b < 2; ++b)
        bf[b] = *reinterpret_cast<const f32x4*>(&sB[cur][(wn * 64 + b * 32 + li) * ROW + 8 * gg + 4 * lh]);
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a][t], bf[b][t], acc[a][b], 0, 0, 0);
    }
    }
    if (kt + 1 < KT) lstore(cur ^ 1);
    __syncthreads();
  }
  // forward scatter: when w % 64 == 0 the wave's 64 rows sit in one image row, so the output
  // pixel of row m0 + wm * 64 + off is a shift of one base pixel (no per-element division)
  const bool rowconst = MODE == 0 && g.w % 64 == 0;
  size_t obase = 0;
  if (rowconst) {
    const int mb = m0 + wm * 64;
    const int bb = mb / hw, rem = mb - bb * hw, y = rem / g.w, x = rem - y * g.w;
    obase = ((size_t)bb * 2 * g.h + 2 * y) * (2 * g.w) + 2 * x;
  }
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int n = n0 + wn * 64 + b * 32 + li;
    if (n >= g.N) continue;
    int o = n, di = 0, dj = 0;
    float bias = 0.f;
    if (MODE == 0) {
      const int ij = n / g.cout;
      o = n - ij * g.cout;
      di = ij >> 1;
      dj = ij & 1;
      bias = g.bias ? g.bias[o] : 0.f;
    }
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m >= g.M) continue;
        float v = acc[a][b][r];
        if constexpr (H3) v = v * (1.f / ua[wave_a(a, r)]) * (1.f / ub[wave_b(b)]);  // exact powers of two
        if (MODE == 0) {
          size_t pix;
          if (rowconst) {
            pix = obase + (size_t)di * (2 * g.w) + 2 * (a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh) + dj;
          } else {
            const int bb = m / hw, rem = m - bb * hw, y = rem / g.w, x = rem - y * g.w;
            pix = ((size_t)bb * 2 * g.h + 2 * y + di) * (2 * g.w) + 2 * x + dj;
          }
          g.dst[pix * g.ldd + o] = v + bias;
        } else {
          if (g.flags & PIS_MASK) v = g.mask[(size_t)m * g.ldm + n] > 0.f ? v : 0.f;
          float* d = g.dst + (size_t)m * g.ldd + n;
          if (g.flags & PIS_ACCUMULATE) v += *d;
          *d = v;
        }
      }
  }
}

// K-step-32 fp16x3 form (pis_tune key 13 = 4, default): gemm_nt_h3_bk32_kernel's pipeline — ONE LDS
// buffer of hi / lo planes ([row][32] fp16, x6w8_off swizzle), the loads of K-step kt + 2 issued
// right after K-step kt + 1 is stored so they land during a whole 24-MFMA phase (the K-step-16
// double buffer above keeps a quarter of the bytes in flight and waits on every K-step: the
// shallow, HBM-bound transposed convs ran at 2.4-2.6 TB/s) — with the transposed conv's
// addressing: the input gradient gathers a 32-wide K chunk of one tap (Cout % 32 == 0); the
// epilogue goes through LDS per wave (32 rows x 64 columns at a time) so every lane finishes 4
// consecutive channels of a pixel with 16-B accesses (forward: the 2 x 2 scatter, whole
// 256-B pixel runs, + bias; input gradient: ReLU mask, accumulate). Needs M, N % 128, w % 32,
// 16-B aligned operands and channel strides % 4 (launch_convt_gemm checks, else key 13 = 3).
template <int MODE>
__global__ __launch_bounds__(256, 3) void convt_h3_kernel(ConvtGemmArgs g) {
  constexpr int BM = 128, BN = 128, BK = 32, KP = 32, AL = BM * 8 / 256, BL = BN * 8 / 256;
  __shared__ __attribute__((aligned(16))) _Float16 smem[2 * (BM + BN) * KP];  // 32 KB: planes, then epilogue
  __shared__ __attribute__((aligned(16))) float sscale[2][4];                // [A|B][staging wave]
  _Float16(*sA)[BM * KP] = reinterpret_cast<_Float16(*)[BM * KP]>(smem);
  _Float16(*sB)[BN * KP] = reinterpret_cast<_Float16(*)[BN * KP]>(smem + 2 * BM * KP);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, lh = lane >> 5;
  const int ntn = g.N / BN;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (bid / ntn) * BM, n0 = (bid % ntn) * BN;
  const int q8 = (tid & 7) * 4;
  const int hw = g.h * g.w;
  // element offset of each staged A row (dgrad: of its 2x2 block's top-left pixel); forward rows
  // are 32 apart: one base
  int64_t arow[MODE == 0 ? 1 : AL];
  if (MODE == 0) {
    arow[0] = (int64_t)(m0 + tid / 8) * g.lda;
  } else {
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int m = m0 + tid / 8 + 32 * i;
      const int b = m / hw, rem = m - b * hw, y = rem / g.w, x = rem - y * g.w;
      arow[MODE == 0 ? 0 : i] = (((int64_t)b * 2 * g.h + 2 * y) * (2 * g.w) + 2 * x) * g.lda;
    }
  }
  f32x4 ra[AL], rb[BL];
  auto gload = [&](int k0) {
    int64_t off = k0 + q8;
    if (MODE == 1) {  // k = (2 di + dj) Cout + o
      const int ij = k0 / g.cout;
      off = ((int64_t)(ij >> 1) * (2 * g.w) + (ij & 1)) * g.lda + (k0 - ij * g.cout) + q8;
    }
#pragma unroll
    for (int i = 0; i < AL; ++i)
      ra[i] = *reinterpret_cast<const f32x4*>(g.a + (MODE == 0 ? arow[0] + (int64_t)(32 * i) * g.lda : arow[MODE == 0 ? 0 : i]) + off);
#pragma unroll
    for (int i = 0; i < BL; ++i)
      rb[i] = *reinterpret_cast<const f32x4*>(g.bt + (size_t)(n0 + tid / 8 + 32 * i) * g.K + k0 + q8);
  };
  float sa = 0.f, sb = 0.f, sa_min = __builtin_inff(), sb_min = __builtin_inff();
  auto lstore = [&]() {
    sa = h3_keep(sa, wave_max_nonneg(absmax_x4(ra)), sa_min);
    sb = h3_keep(sb, wave_max_nonneg(absmax_x4(rb)), sb_min);
    if (lane == 0) {
      sscale[0][wave] = sa;
      sscale[1][wave] = sb;
    }
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      u32x2 h, l;
      split2h_x4(ra[i] * sa, h, l);
      const int o = x6w8_off(tid / 8 + 32 * i, q8 >> 3) + (q8 & 7);
      *reinterpret_cast<u32x2*>(&sA[0][o]) = h;
      *reinterpret_cast<u32x2*>(&sA[1][o]) = l;
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      u32x2 h, l;
      split2h_x4(rb[i] * sb, h, l);
      const int o = x6w8_off(tid / 8 + 32 * i, q8 >> 3) + (q8 & 7);
      *reinterpret_cast<u32x2*>(&sB[0][o]) = h;
      *reinterpret_cast<u32x2*>(&sB[1][o]) = l;
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const int KT = g.K / BK;
  gload(0);
  lstore();
  if (KT > 1) gload(BK);
  __syncthreads();
  f32x4 ua = {1.f, 1.f, 1.f, 1.f};  // accumulator units: A scale per row group r >> 2, B scale of the column
  float ub = 1.f;
  for (int kt = 0; kt < KT; ++kt) {
    const f32x4 na = *reinterpret_cast<const f32x4*>(&sscale[0][0]);
    const float nb = sscale[1][(li >> 3) & 3];
    if (kt == 0) {
      ua = na;
      ub = nb;
    } else if (na[0] != ua[0] || na[1] != ua[1] || na[2] != ua[2] || na[3] != ua[3] || nb != ub) {
      const float rb_ = nb / ub;
      float f[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) f[q] = na[q] / ua[q] * rb_;
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[a][b][r] *= f[r >> 2];
      ua = na;
      ub = nb;
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f16x8 af[2][2], bf[2][2];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
          af[p][a] = *reinterpret_cast<const f16x8*>(&sA[p][x6w8_off(wm * 64 + a * 32 + li, 2 * ks + lh)]);
#pragma unroll
        for (int b = 0; b < 2; ++b)
          bf[p][b] = *reinterpret_cast<const f16x8*>(&sB[p][x6w8_off(wn * 64 + b * 32 + li, 2 * ks + lh)]);
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {  // smallest partial products first
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1][a], bf[0][b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0][a], bf[1][b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0][a], bf[0][b], acc[a][b], 0, 0, 0);
        }
    }
    if (kt + 1 < KT) {
      __syncthreads();
      lstore();
      __syncthreads();
      if (kt + 2 < KT) gload((kt + 2) * BK);
    }
  }
  // epilogue through LDS: wave's [32 rows][64 columns] fp32 image (8 KB of the 32 KB planes), one
  // 32-row half (a) at a time; a 32-row run of pixels lies in one image row (w % 32 == 0)
  float inv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) inv[q] = 1.f / (ua[q] * ub);  // exact powers of two
  float* E = reinterpret_cast<float*>(smem) + wave * (32 * 64);
  const int c4 = 4 * (lane & 15);
  const int nb0 = n0 + wn * 64 + c4;  // this lane's 4 columns
  int o = nb0, di = 0, dj = 0;
  f32x4 bias4 = {0.f, 0.f, 0.f, 0.f};
  if (MODE == 0) {
    const int ij = nb0 / g.cout;
    o = nb0 - ij * g.cout;
    di = ij >> 1;
    dj = ij & 1;
    if (g.bias) bias4 = *reinterpret_cast<const f32x4*>(g.bias + o);
  }
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    __syncthreads();  // the K loop's last fragment reads (a = 0) / the previous half's reads (a = 1)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r)
        E[((r & 3) + 8 * (r >> 2) + 4 * lh) * 64 + b * 32 + li] = acc[a][b][r] * inv[r >> 2];
    __syncthreads();
    const int mb = m0 + wm * 64 + a * 32;  // first row of the half
    size_t obase = 0;
    if (MODE == 0) {
      const int bb = mb / hw, rem = mb - bb * hw, y = rem / g.w, x = rem - y * g.w;
      obase = ((size_t)bb * 2 * g.h + 2 * y + di) * (2 * g.w) + 2 * x + dj;
    }
    f32x4 mk[8], old[8];
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int rl = 4 * p + (lane >> 4);
      mk[p] = f32x4{1.f, 1.f, 1.f, 1.f};
      old[p] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (MODE == 1) {
        if (g.flags & PIS_MASK) mk[p] = *reinterpret_cast<const f32x4*>(g.mask + (size_t)(mb + rl) * g.ldm + nb0);
        if (g.flags & PIS_ACCUMULATE) old[p] = *reinterpret_cast<const f32x4*>(g.dst + (size_t)(mb + rl) * g.ldd + nb0);
      }
    }
#pragma unroll
    for (int p = 0; p < 8; ++p) {
      const int rl = 4 * p + (lane >> 4);
      f32x4 v = *reinterpret_cast<const f32x4*>(&E[rl * 64 + c4]);
      if (MODE == 0) {
        *reinterpret_cast<f32x4*>(g.dst + (obase + 2 * (size_t)rl) * g.ldd + o) = v + bias4;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (mk[p][e] > 0.f ? v[e] : 0.f) + old[p][e];
        *reinterpret_cast<f32x4*>(g.dst + (size_t)(mb + rl) * g.ldd + nb0) = v;
      }
    }
  }
}

// 0 = handled, 1 = shape not covered (caller falls back to the implicit GEMM)
int launch_convt_gemm(int mode, const float* a, int lda, const float* bt, int B, int h, int w, int cin, int cout,
                      const float* bias, const float* mask, int ldm, float* dst, int ldd, int flags,
                      hipStream_t s) {
  if (tune_get(PIS_TUNE_CONVT_GEMM) == 0 || cin % 16 || cout % 16 || lda % 4) return 1;
  ConvtGemmArgs g{};
  g.a = a; g.lda = lda; g.bt = bt; g.B = B; g.h = h; g.w = w; g.cin = cin; g.cout = cout;
  g.M = B * h * w;
  g.N = mode == 0 ? 4 * cout : cin;
  g.K = mode == 0 ? cin : 4 * cout;
  g.bias = bias; g.mask = mask; g.ldm = ldm; g.dst = dst; g.ldd = ldd; g.flags = flags;
  const int grid = (int)(cdiv(g.M, 128) * cdiv(g.N, 128));
  int v = tune_get(PIS_TUNE_CONVT_GEMM);
  if (v == 4) {
    auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    const bool ok = g.M % 128 == 0 && g.N % 128 == 0 && w % 32 == 0 && cout % 32 == 0 && cin % 32 == 0 &&
                    lda % 4 == 0 && ldd % 4 == 0 && a16(a) && a16(bt) && a16(dst) &&
                    (mode == 0 ? (!bias || a16(bias)) : (!(flags & PIS_MASK) || (a16(mask) && ldm % 4 == 0)));
    if (ok) {
      if (mode == 0) hipLaunchKernelGGL(convt_h3_kernel<0>, dim3(grid), dim3(256), 0, s, g);
      else hipLaunchKernelGGL(convt_h3_kernel<1>, dim3(grid), dim3(256), 0, s, g);
      return launch_status(mode == 0 ? "convt_h3_fwd" : "convt_h3_dgrad");
    }
    v = 3;
  }
  const int ar = v == 1 ? 1 : v == 3 ? 2 : 0;  // 2 = fp32 MFMA
  if (mode == 0 && ar == 2) hipLaunchKernelGGL((convt_gemm_kernel<0, 2>), dim3(grid), dim3(256), 0, s, g);
  else if (mode == 0 && ar == 1) hipLaunchKernelGGL((convt_gemm_kernel<0, 1>), dim3(grid), dim3(256), 0, s, g);
  else if (mode == 0) hipLaunchKernelGGL((convt_gemm_kernel<0, 0>), dim3(grid), dim3(256), 0, s, g);
  else if (ar == 2) hipLaunchKernelGGL((convt_gemm_kernel<1, 2>), dim3(grid), dim3(256), 0, s, g);
  else if (ar == 1) hipLaunchKernelGGL((convt_gemm_kernel<1, 1>), dim3(grid), dim3(256), 0, s, g);
  else hipLaunchKernelGGL((convt_gemm_kernel<1, 0>), dim3(grid), dim3(256), 0, s, g);
  return launch_status(mode == 0 ? "convt_gemm_fwd" : "convt_gemm_dgrad");
}

}  // namespace pis
