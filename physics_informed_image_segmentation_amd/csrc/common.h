// Shared helpers for the gfx950 kernels behind the pis_* C-ABI.
// Conventions (include/pis_capi.h): every entry point returns 0 or a negative
// code, never throws, never allocates, never synchronises; it launches on the
// caller's stream. pis_last_error() returns the last message of this thread.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <algorithm>

#include "../../include/pis_capi.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace pis {

void set_error(const char* fmt, ...);
int tune_get(int key);  // pis_tune() knob value (csrc/capi.hip)

// Optional host callback around the heavy launches (pis_set_launch_hook): lets a
// profiler record HIP events on the launch stream right before/after one kernel.
void launch_hook(const char* kernel, int phase, hipStream_t s, double flop);
void gemm_done(hipStream_t s);  // records the event armed by pis_arm_gemm_event, if any

inline int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return PIS_ERR_LAUNCH;
  }
  return PIS_OK;
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Bijective XCD-aware remap (cdna_hip_programming.md §5 'XCD swizzle must be
// bijective'): blocks dealt round-robin over 8 XCDs get consecutive logical
// ids per XCD, so neighbouring tiles share an L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = bid % 8, loc = bid / 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

// The same over a 2-D grid of gridDim.y independent batches of gridDim.x blocks: the dispatcher
// deals the flattened ids (x fastest) round-robin over the XCDs, so remapping the flattened id
// gives each XCD runs of consecutive (batch, block) pairs — whole tile groups of one batch that
// share operand rows in that XCD's L2 — instead of an eighth of every batch's blocks
struct Remap2 {
  int batch, bid;
};
__device__ __forceinline__ Remap2 xcd_remap2() {
  const int gx = gridDim.x;
  const int l = xcd_remap(blockIdx.y * gx + blockIdx.x, gx * gridDim.y);
  return Remap2{l / gx, l % gx};
}

// 16-bit element offset of 16-B chunk `chunk` (0..3) of row `row` in [row][32] LDS images, the
// chunk XOR-swizzled by row bits 2..3: conflict-free ds_read_b128 fragments AND ds_write_b64 staging
__device__ __forceinline__ int x6w8_off(int row, int chunk) { return row * 32 + 8 * (chunk ^ ((row >> 2) & 3)); }

// ---- bf16x6: exact 3-way bf16 split of fp32 operands ------------------------
// hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid); both subtractions are exact, and
// hi + mid + lo == x (24 significant bits). Two values per step: one v_cvt_pk_bf16_f32 per level,
// the bf16 pair widened back to fp32 by a shift / mask, one v_pk_add_f32 per residual (4.5 VALU
// per value). Outputs are packed bf16 pairs (element 0 in the low half, memory order).
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 pis_bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split3_pair(f32x2 x, unsigned& h, unsigned& m, unsigned& l) {
  const unsigned hu = __builtin_bit_cast(unsigned, __builtin_convertvector(x, pis_bf16x2));
  const f32x2 r = x - f32x2{__builtin_bit_cast(float, hu << 16), __builtin_bit_cast(float, hu & 0xffff0000u)};
  const unsigned mu = __builtin_bit_cast(unsigned, __builtin_convertvector(r, pis_bf16x2));
  const f32x2 r2 = r - f32x2{__builtin_bit_cast(float, mu << 16), __builtin_bit_cast(float, mu & 0xffff0000u)};
  h = hu;
  m = mu;
  l = __builtin_bit_cast(unsigned, __builtin_convertvector(r2, pis_bf16x2));
}

// four values -> three planes of 4 bf16 (8 bytes each)
__device__ __forceinline__ void split3_x4(f32x4 v, u32x2& h, u32x2& m, u32x2& l) {
  unsigned h0, m0, l0, h1, m1, l1;
  split3_pair(f32x2{v[0], v[1]}, h0, m0, l0);
  split3_pair(f32x2{v[2], v[3]}, h1, m1, l1);
  h = u32x2{h0, h1};
  m = u32x2{m0, m1};
  l = u32x2{l0, l1};
}

// ---- fp16x3: x = (hi + lo) / s with hi = fp16(x s), lo = fp16(x s - hi), s a power
// of two per wave and K-step; the three products lo*hi, hi*lo, hi*hi on fp16 MFMA
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2_t __attribute__((ext_vector_type(2)));
// hi: v_cvt_pk_f16_f32 per pair; lo: one v_fma_mix{lo,hi}_f16 per value, fp16(v - hi) with the
// fp16 hi read straight from its half of the packed register (1.5 VALU per value; widening hi back
// to fp32 first took 2.5). The residual v - hi is exact in fp32 (v has 24 significant bits, hi
// its leading 11), so rounding it once to fp16 inside the fma gives the same lo as the widened form.
__device__ __forceinline__ void split2h_x4(f32x4 v, u32x2& h, u32x2& l) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  const f2 a = {v[0], v[1]}, b = {v[2], v[3]};
  const unsigned ha = __builtin_bit_cast(unsigned, __builtin_convertvector(a, f16x2_t));
  const unsigned hb = __builtin_bit_cast(unsigned, __builtin_convertvector(b, f16x2_t));
  unsigned la, lb;
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(la) : "v"(v[0]), "v"(ha));
  asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(la) : "v"(v[1]), "v"(ha));
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(lb) : "v"(v[2]), "v"(hb));
  asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(lb) : "v"(v[3]), "v"(hb));
  h = u32x2{ha, hb};
  l = u32x2{la, lb};
}

// 2^(13 - e) for m in [2^e, 2^(e+1)): m * scale lands in [2^13, 2^14), 4x under fp16's largest
// finite value; 1 for a zero (or NaN) tile, 2^127 for a tile below 2^-114
__device__ __forceinline__ float h3_scale(float m) {
  if (!(m > 0.f)) return 1.f;
  const int eb = (int)(__float_as_uint(m) >> 23);  // m >= 0: the biased exponent
  const int sb = 267 - eb;                           // 127 + 13 - (eb - 127)
  return __uint_as_float((unsigned)(sb > 254 ? 254 : sb) << 23);
}

// the scale for a tile of max m given the current scale: kept while m * cur stays in [2^7, 2^15)
// (fp16 digits for everything above 2^-10 of the max, 2x headroom), so accumulators are rarely
// rescaled; else re-chosen (h3_scale). cur = 0 always re-chooses; an all-zero K-step keeps cur.
// smin (per wave, +inf before the first K-step) is the smallest scale used so far, i.e. the one
// of the largest operands the accumulators hold: a scale may rise at most 2^32 above it. The
// accumulators are re-expressed in every new scale, so without the cap a K-step of operands
// 2^100 below the earlier ones would multiply partial sums of ~2^26 by ~2^200 (inf, for good);
// with it they stay below K 2^90, and the capped K-step's operands — at most 2^-32 of the sum
// already accumulated — keep fp16 digits down to 2^-46 of it.
__device__ __forceinline__ float h3_keep(float cur, float m, float& smin) {
  if (!(m > 0.f)) return cur > 0.f ? cur : 1.f;
  const float v = m * cur;
  // wave-uniform: kept in SGPRs (the GEMMs run at their VGPR limit)
  const float s = __int_as_float(__builtin_amdgcn_readfirstlane(
      __float_as_int(fminf((v >= 128.f && v < 32768.f) ? cur : h3_scale(m), smin * 0x1p32f))));
  smin = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(fminf(smin, s))));
  return s;
}

// 4 consecutive fp16 of one LDS row (8-B aligned) read transposed across the 16-lane group
// (ds_read_b64_tr_b16): lane (4 q + p) of the group addresses row q, columns 4 p .. 4 p + 3 of a
// 4 x 16 block; lane j of the group receives column j, rows 0..3
typedef short s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ s16x4 tr_read(const _Float16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

template <int CTRL, int RMASK>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, RMASK, 0xf, true));
}
// max |x| over the 4 N values of x (>= 0): one v_max3_f32 with |.| source modifiers per pair.
// Written out because fmaxf chains get a quieting v_max per operand (maxnum canonicalization) and
// only partly fuse into v_max3; a quiet NaN operand is skipped as fmaxf would skip it.
template <int N>
__device__ __forceinline__ float absmax_x4(const f32x4 (&x)[N]) {
  float m = 0.f;
#pragma unroll
  for (int i = 0; i < 4 * N; i += 2)
    asm("v_max3_f32 %0, |%1|, |%2|, %0" : "+v"(m) : "v"(x[i >> 2][i & 3]), "v"(x[i >> 2][(i & 3) + 1]));
  return m;
}

// max over a wave of v >= 0 (DPP row shifts + row broadcasts: VALU only, no LDS round trip),
// returned uniform
template <int N, int M>
__device__ __forceinline__ float absmax_x4(const f32x4 (&x)[N][M]) {
  float m = 0.f;
#pragma unroll
  for (int i = 0; i < N; ++i)
#pragma unroll
    for (int j = 0; j < M; ++j) {
      asm("v_max3_f32 %0, |%1|, |%2|, %0" : "+v"(m) : "v"(x[i][j][0]), "v"(x[i][j][1]));
      asm("v_max3_f32 %0, |%1|, |%2|, %0" : "+v"(m) : "v"(x[i][j][2]), "v"(x[i][j][3]));
    }
  return m;
}

// (on the bit patterns: for v >= 0, NaN-free, unsigned order is float order, and integer max
// has no maxnum canonicalization, so each step is one v_max_u32 with the DPP folded in)
template <int CTRL, int RMASK>
__device__ __forceinline__ unsigned dpp_u(unsigned x) {
  return (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, RMASK, 0xf, true);
}
__device__ __forceinline__ float wave_max_nonneg(float f) {
  unsigned v = __float_as_uint(f);
  v = max(v, dpp_u<0x111, 0xf>(v));  // row_shr:1
  v = max(v, dpp_u<0x112, 0xf>(v));  // row_shr:2
  v = max(v, dpp_u<0x114, 0xf>(v));  // row_shr:4
  v = max(v, dpp_u<0x118, 0xf>(v));  // row_shr:8: lane 15 of each row holds the row's max
  v = max(v, dpp_u<0x142, 0xa>(v));  // row_bcast:15
  v = max(v, dpp_u<0x143, 0xc>(v));  // row_bcast:31: lane 63 holds the wave's max
  return __uint_as_float(__builtin_amdgcn_readlane(v, 63));
}

// 16-byte load from a wave-uniform base (SGPRs) at an unsigned 32-bit per-lane byte offset, as a
// raw buffer load: the address needs no per-lane 64-bit arithmetic (offsets below 2 GiB)
__device__ __forceinline__ u32x4 buf_load16(const void* base, uint32_t off) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
  return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// max of v >= 0 over each aligned group of 8 lanes, returned in every lane of the group (two quad
// permutes + row_half_mirror)
__device__ __forceinline__ float group8_max_nonneg(float f) {
  unsigned v = __float_as_uint(f);    // bit-pattern max, as wave_max_nonneg
  v = max(v, dpp_u<0xB1, 0xf>(v));   // quad_perm [1,0,3,2]
  v = max(v, dpp_u<0x4E, 0xf>(v));   // quad_perm [2,3,0,1]
  v = max(v, dpp_u<0x141, 0xf>(v));  // row_half_mirror: the other quad of the 8
  return __uint_as_float(v);
}

// the fp16x3 scale s = 2^(13 - e) for a group max m in [2^e, 2^(e+1)) (as h3_scale) and its exact
// inverse; s is capped at 2^126 so that 1/s stays a normal float; s = inv = 1 for a zero / NaN max
__device__ __forceinline__ void h2_scale_pair(float m, float& s, float& inv) {
  // selects, not branches: this runs in fully unrolled loops where a divergent branch would cut
  // the schedule into pieces
  const bool ok = m > 0.f;
  const int eb = (int)(__float_as_uint(m) >> 23) & 0xff;
  const int sb = std::min(267 - eb, 253);
  s = ok ? __uint_as_float((unsigned)sb << 23) : 1.f;
  inv = ok ? __uint_as_float((unsigned)(254 - sb) << 23) : 1.f;
}

// LDS element offset of (row, k) in a [row][16 k] bf16 plane: the two 16-B chunks of a row are
// swapped on rows where bit 2 ^ bit 3 of the row is set, so the 16 rows a ds_read_b128 lane group
// reads at one chunk hit 16 distinct slots of the 256-B bank row, and 8 consecutive rows written
// by a ds_write_b128 group hit 8 distinct slots of the 128-B write bank row (unswizzled 32-B rows:
// 2-way on both)
__device__ __forceinline__ int wsw(int row, int k) {
  return row * 16 + ((((k >> 3) ^ ((row >> 2) ^ (row >> 3))) & 1) << 3) + (k & 7);
}

// sum of v over each aligned group of 16 lanes (a DPP row), returned in every lane of the group:
// xor-1 and xor-2 quad permutes, then row_half_mirror (lane i <-> 7 - i) and row_mirror (i <-> 15 - i).
// VALU only (no LDS traffic, unlike a 16-wide __shfl_xor); every lane's result is the same bits
__device__ __forceinline__ float group16_sum(float v) {
  v += dpp_f<0xB1, 0xf>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E, 0xf>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141, 0xf>(v);  // row_half_mirror
  v += dpp_f<0x140, 0xf>(v);  // row_mirror
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

}  // namespace pis

#define PIS_CHECK_ARG(cond, ...)      \
  do {                                \
    if (!(cond)) {                    \
      pis::set_error(__VA_ARGS__);    \
      return PIS_ERR_ARG;             \
    }                                 \
  } while (0)
