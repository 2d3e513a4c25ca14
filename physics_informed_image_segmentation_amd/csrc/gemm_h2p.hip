// Batched NT GEMM on PRE-SPLIT fp16x3 operands (the Winograd F(4x4,3x3) contractions' candidate
// successor to gemm_nt_h3_bk32_kernel):
//   C[b][m][n] = ia[b][m] ib[b][n] sum_k (Ah Bh + Ah Bl + Al Bh)[b][m|n][k]
// where Ah / Al (Bh / Bl) are the hi / lo fp16 planes of the fp32 operand row times a power-of-two
// row scale s (ia = 1 / s), split ONCE by the operand's producer instead of once per block that
// reads it. The kernel is then a plain fp16 MFMA GEMM: both operands arrive global -> LDS by
// LDS-DMA (global_load_lds_dwordx4, no VGPR staging, no split VALU, no per-K-step scale logic),
// 128 x 128 tile, 4 waves of 64 x 64 (2 x 2 v_mfma_f32_32x32x16_f16 tiles, three products per
// fragment pair, smallest first), K-steps of 32 through two 32-KB LDS stages (2 blocks per CU).
// The unscaling is two exact power-of-two multiplies per output in the epilogue.
// Requirements: M, N % 128 == 0, K % 32 == 0, 16-B aligned planes.
#include "common.h"
#include "igemm.h"

namespace pis {

constexpr int HP_BK = 32;                    // halves per K-step
constexpr int HP_PLANE = 128 * HP_BK;        // halves per plane per stage (8 KB)
constexpr int HP_STAGE = 4 * HP_PLANE;       // Ah, Al, Bh, Bl (32 KB)

// [row][32] fp16 images, 16-B chunk XOR-swizzled by row bits 2..3 (x6w8_off): conflict-free
// ds_read_b128 fragment reads; the LDS-DMA writes stay lane-linear and the swizzle is applied to
// their SOURCE addresses (cdna_hip_programming.md rule 21)
__global__ __launch_bounds__(256, 2) void gemm_h2p_kernel(H2pArgs g) {
  __shared__ __attribute__((aligned(16))) _Float16 smem[2 * HP_STAGE];
  const Remap2 rm = xcd_remap2();
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, lh = lane >> 5;
  const int ntn = g.N / 128;
  const int m0 = (rm.bid / ntn) * 128, n0 = (rm.bid % ntn) * 128;
  const int KT = g.K / HP_BK;
  // wave w fills plane w (0 Ah, 1 Al, 2 Bh, 3 Bl) of a stage: 8 pieces of 16 rows x 64 B; lane l of
  // piece i lands at row 16 i + l / 4, physical chunk l % 4 and loads the logical chunk there
  const _Float16* src;
  {
    const _Float16* planes[4] = {g.ah, g.al, g.bh, g.bl};
    const int64_t bs = wave < 2 ? g.bsa : g.bsb;
    const int r0 = wave < 2 ? m0 : n0;
    src = planes[wave] + rm.batch * bs + (size_t)r0 * g.K;
  }
  const int prow = lane >> 2, pslot = lane & 3;
  auto issue = [&](int kt, int st) __attribute__((always_inline)) {
    _Float16* base = smem + st * HP_STAGE + wave * HP_PLANE;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int row = 16 * i + prow, c = pslot ^ ((row >> 2) & 3);
      const _Float16* gp = src + (size_t)row * g.K + kt * HP_BK + 8 * c;
      __builtin_amdgcn_global_load_lds(gp, (__attribute__((address_space(3))) void*)(base + 512 * i), 16, 0, 0);
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  // the epilogue's inverse row scales, loaded before the K loop (their latency hides under it)
  float sa[2][16], sb[2];
  {
    const float* ia = g.ia + rm.batch * g.bsia;
    const float* ib = g.ib + rm.batch * g.bsib;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) sa[a][r] = ia[m0 + wm * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh];
#pragma unroll
    for (int b = 0; b < 2; ++b) sb[b] = ib[n0 + wn * 64 + b * 32 + li];
  }

  issue(0, 0);
  for (int kt = 0; kt < KT; ++kt) {
    __syncthreads();  // K-step kt has landed (vmcnt(0)); every wave is done with the other stage
    if (kt + 1 < KT) issue(kt + 1, (kt + 1) & 1);
    const _Float16* st = smem + (kt & 1) * HP_STAGE;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = 2 * ks + lh;  // this lane's 8 K values: logical chunk ch of its row
      f16x8 af[2][2], bf[2][2];    // [hi | lo][tile]
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int r = wm * 64 + a * 32 + li;
        af[0][a] = *reinterpret_cast<const f16x8*>(st + 0 * HP_PLANE + x6w8_off(r, ch));
        af[1][a] = *reinterpret_cast<const f16x8*>(st + 1 * HP_PLANE + x6w8_off(r, ch));
      }
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int r = wn * 64 + b * 32 + li;
        bf[0][b] = *reinterpret_cast<const f16x8*>(st + 2 * HP_PLANE + x6w8_off(r, ch));
        bf[1][b] = *reinterpret_cast<const f16x8*>(st + 3 * HP_PLANE + x6w8_off(r, ch));
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
  }
  float* C = g.c + rm.batch * g.bsc;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int n = n0 + wn * 64 + b * 32 + li;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        C[(size_t)m * g.N + n] = (acc[a][b][r] * sa[a][r]) * sb[b];
      }
  }
}

int launch_gemm_h2p(const H2pArgs& g, int batch, hipStream_t s) {
  if (g.M % 128 || g.N % 128 || g.K % HP_BK || g.K <= 0)
    return set_error("gemm_h2p: needs M, N % 128 == 0 and K % 32 == 0"), PIS_ERR_ARG;
  const dim3 grid((g.M / 128) * (g.N / 128), batch);
  hipLaunchKernelGGL(gemm_h2p_kernel, grid, dim3(256), 0, s, g);
  return launch_status("gemm_h2p");
}

// rows of X (fp32 [batch][rows][K], K % 4 == 0) -> hi / lo fp16 planes of x s_row and 1 / s_row,
// s_row = h3_scale(max |row|) (the max lands in [2^13, 2^14)); one wave per row (tooling and tests:
// the producers of the Winograd operands split their own rows)
__global__ __launch_bounds__(256) void split_rows_h2_kernel(const float* __restrict__ X, int rows, int K,
                                                            _Float16* __restrict__ hi, _Float16* __restrict__ lo,
                                                            float* __restrict__ inv, int64_t nrows_total) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= nrows_total) return;
  const float* x = X + row * K;
  float m = 0.f;
  for (int k = 4 * lane; k < K; k += 256) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(x + k);
    m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
  }
  const float s = h3_scale(__int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(wave_max_nonneg(m)))));
  for (int k = 4 * lane; k < K; k += 256) {
    u32x2 h, l;
    split2h_x4(*reinterpret_cast<const f32x4*>(x + k) * s, h, l);
    *reinterpret_cast<u32x2*>(hi + row * K + k) = h;
    *reinterpret_cast<u32x2*>(lo + row * K + k) = l;
  }
  if (lane == 0) inv[row] = 1.f / s;
  (void)rows;
}

int launch_split_rows_h2(const float* X, int64_t nrows, int K, _Float16* hi, _Float16* lo, float* inv,
                         hipStream_t s) {
  if (K % 4) return set_error("split_rows_h2: K % 4 != 0"), PIS_ERR_ARG;
  hipLaunchKernelGGL(split_rows_h2_kernel, dim3((unsigned)cdiv(nrows, 4)), dim3(256), 0, s, X, 0, K, hi, lo, inv,
                     nrows);
  return launch_status("split_rows_h2");
}

}  // namespace pis

using namespace pis;

// Tooling (tools/bench_gemm.py variant 20): split A ([batch][M][K]) and B ([batch][N][K]) by rows into
// the planes of ws (untimed by the caller when `split` is 1), then run the pre-split GEMM only
// (`split` 0 reuses the planes of the previous call). ws >= 4 (M + N) K batch bytes + 4 (M + N) batch.
extern "C" int pis_debug_gemm_h2p(const float* A, const float* B, float* C, int M, int N, int K, int batch, void* ws,
                                  size_t ws_bytes, int split, pis_stream_t stream) {
  PIS_CHECK_ARG(A && B && C && ws && M > 0 && N > 0 && K > 0 && batch > 0, "pis_debug_gemm_h2p: bad arguments");
  const size_t na = (size_t)batch * M * K, nb = (size_t)batch * N * K;
  PIS_CHECK_ARG(ws_bytes >= 4 * (na + nb) + 4 * (size_t)batch * (M + N) + 64, "pis_debug_gemm_h2p: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  _Float16* ah = (_Float16*)ws;
  _Float16* al = ah + na;
  _Float16* bh = al + na;
  _Float16* bl = bh + nb;
  float* ia = (float*)(bl + nb);
  float* ib = ia + (size_t)batch * M;
  if (split) {
    int rc = launch_split_rows_h2(A, (int64_t)batch * M, K, ah, al, ia, s);
    if (!rc) rc = launch_split_rows_h2(B, (int64_t)batch * N, K, bh, bl, ib, s);
    if (rc) return rc;
  }
  H2pArgs g{};
  g.ah = ah; g.al = al; g.bh = bh; g.bl = bl; g.ia = ia; g.ib = ib; g.c = C;
  g.M = M; g.N = N; g.K = K;
  g.bsa = (int64_t)M * K; g.bsb = (int64_t)N * K; g.bsc = (int64_t)M * N; g.bsia = M; g.bsib = N;
  return launch_gemm_h2p(g, batch, s);
}
