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
int reduce_slabs2(const float* part, int splits, int64_t n, float* dst, const float* part_b, int splits_b,
                  int64_t n_b, float* dst_b, int accumulate, hipStream_t s);

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
// sample; its threads tile a row with float4 columns (TX = min(W/4, 256) threads a row) and
// split the rows into RY = 256/TX contiguous segments. Each thread walks its segment DOWN its
// column with a sliding window of three u rows in registers, so a row of u is loaded once per
// thread (not three times): per U rows it issues U u-rows, U t-rows and the 2U left/right ghost
// scalars (reflect: column -1 is column 1, W is W-2; re-reads of lines the block fetches, L1/L2
// hits) before any arithmetic. No LDS staging, no integer division in the loop. A one-block
// finalize launch reduces the per-block partials in a fixed order: deterministic.
// ---------------------------------------------------------------------------
constexpr int LOSS_ROW_BATCH = 2;  // rows per thread per batch of the whole-row forward

struct LossRowArgs {
  LossArgs g;
  int rows;             // image rows per block
  int bands;            // blocks per sample
  float* terms;
  int* counts;
  float* scores;
};

template <bool RD, bool PF>
__global__ __launch_bounds__(256, 5) void loss_fwd_rows_kernel(LossRowArgs a) {
  constexpr bool ST = RD || PF;
  const LossArgs& g = a.g;
  const int H = g.H, W = g.W, W4 = W >> 2;
  const int band = blockIdx.x, b = blockIdx.y;
  const int y0 = band * a.rows, nr = min(a.rows, H - y0);
  const float* u = g.p + (size_t)b * H * W;
  const float* tt = g.t + (size_t)b * H * W;
  const int TX = min(W4, 256), RY = 256 / TX;
  const int tx = threadIdx.x % TX, ty = threadIdx.x / TX;
  const int seg = (nr + RY - 1) / RY;
  const int ys = y0 + ty * seg, ye = min(ys + seg, y0 + nr);  // ys >= ye: an idle thread
  constexpr float kLn2 = 0.69314718055994531f, kClamp2 = -144.26950408889634f;  // -100 / ln 2
  // per-thread sums as pixel pairs (packed fp32 math: one v_pk_* instruction per two pixels)
  f32x2 s_it = {0.f, 0.f}, s_p = s_it, s_t = s_it, s_bce2 = s_it, s_rd = s_it, s_g2 = s_it, s_q2 = s_it;
  int c_i = 0, c_p = 0, c_t = 0;
  // Two rows per batch (LOSS_ROW_BATCH); the NEXT batch's loads are issued before this batch's
  // arithmetic (software pipelining: each wave keeps a batch in flight while it computes). Every
  // value is a named register: arrays indexed by a loop variable are promoted to LDS by the
  // compiler before unrolling.
  struct Batch {
    f32x4 d0, d1;            // ST: rows y + 1, y + 2 (down neighbours; row H is H-2); else rows y, y + 1
    f32x4 t0, t1;            // targets of rows y, y + 1
    float l0, r0, l1, r1;    // left / right ghosts of rows y, y + 1 (reflect: column -1 is 1, W is W-2)
  };
  for (int xi = tx; xi < W4 && ty < RY && ys < ye; xi += TX) {
    const int xb = 4 * xi;
    const int xl = xb == 0 ? 1 : xb - 1, xr = xb + 4 == W ? W - 2 : xb + 4;
    // 32-bit offsets from the block-uniform sample base (H W < 2^31); rows past the segment repeat
    // its last row (discarded below), so the loads are branch-free
    auto load = [&](Batch& bt, int y) {
      const int ya = min(y, ye - 1), yb = min(y + 1, ye - 1);
      bt.t0 = *(const f32x4*)(tt + (ya * W + xb));
      bt.t1 = *(const f32x4*)(tt + (yb * W + xb));
      if constexpr (ST) {
        bt.d0 = *(const f32x4*)(u + (refl(min(ya + 1, H), H) * W + xb));
        bt.d1 = *(const f32x4*)(u + (refl(min(yb + 1, H), H) * W + xb));
        bt.l0 = u[ya * W + xl];
        bt.r0 = u[ya * W + xr];
        bt.l1 = u[yb * W + xl];
        bt.r1 = u[yb * W + xr];
      } else {
        bt.d0 = *(const f32x4*)(u + (ya * W + xb));
        bt.d1 = *(const f32x4*)(u + (yb * W + xb));
      }
    };
    f32x4 up, cur;  // ST: rows y - 1 and y (reflect: row -1 is row 1)
    if constexpr (ST) {
      up = *(const f32x4*)(u + (refl(ys - 1, H) * W + xb));
      cur = *(const f32x4*)(u + (ys * W + xb));
    }
    const f32x2 a2 = {g.a, g.a}, D2 = {g.D, g.D}, rx2 = {g.rx, g.rx};
    // two pixels: p, t, and the up / down / left / right neighbours of u (packed fp32 math)
    auto px2 = [&](f32x2 p, f32x2 t, f32x2 uu, f32x2 ud, f32x2 ul, f32x2 ur) {
      s_it = __builtin_elementwise_fma(p, t, s_it);
      s_p += p;
      s_t += t;
      // (t - 1) L1 - t L0 = t (L1 - L0) - L1 (log2 domain, clamped at -100 / ln 2)
      const f32x2 l1 = {fmaxf(__builtin_amdgcn_logf(1.f - p.x), kClamp2), fmaxf(__builtin_amdgcn_logf(1.f - p.y), kClamp2)};
      const f32x2 l0 = {fmaxf(__builtin_amdgcn_logf(p.x), kClamp2), fmaxf(__builtin_amdgcn_logf(p.y), kClamp2)};
      s_bce2 = __builtin_elementwise_fma(t, l1 - l0, s_bce2) - l1;
      // thresholded counters as wave ballots: one compare per pixel on the VALU, the counting on
      // the scalar unit (exact; lanes past their segment's end are inactive and count 0)
      const unsigned long long mp0 = __ballot(p.x > g.thr), mt0 = __ballot(t.x > 0.5f);
      const unsigned long long mp1 = __ballot(p.y > g.thr), mt1 = __ballot(t.y > 0.5f);
      c_p += __popcll(mp0) + __popcll(mp1);
      c_t += __popcll(mt0) + __popcll(mt1);
      c_i += __popcll(mp0 & mt0) + __popcll(mp1 & mt1);
      if constexpr (ST) {
        const f32x2 qq = __builtin_elementwise_fma(-p, p, p);  // p (1 - p)
        if (RD) {
          const f32x2 lap = __builtin_elementwise_fma(f32x2{-4.f, -4.f}, p, (uu + ud) + (ul + ur));
          const f32x2 rr = __builtin_elementwise_fma(D2, lap, rx2 * qq * (p - a2));
          s_rd = __builtin_elementwise_fma(rr, rr, s_rd);
        }
        if (PF) {
          const f32x2 gx = ur - ul, gy = ud - uu;  // 2x the central differences
          s_g2 = __builtin_elementwise_fma(gx, gx, __builtin_elementwise_fma(gy, gy, s_g2));
          s_q2 = __builtin_elementwise_fma(qq, qq, s_q2);
        }
      }
    };
    // one row of 4 pixels as pairs (0, 1), (2, 3): c the row, uu / dd the rows above / below
    auto row = [&](f32x4 c, f32x4 t, f32x4 uu, f32x4 dd, float l, float r) {
      px2(f32x2{c.x, c.y}, f32x2{t.x, t.y}, f32x2{uu.x, uu.y}, f32x2{dd.x, dd.y}, f32x2{l, c.x}, f32x2{c.y, c.z});
      px2(f32x2{c.z, c.w}, f32x2{t.z, t.w}, f32x2{uu.z, uu.w}, f32x2{dd.z, dd.w}, f32x2{c.y, c.z}, f32x2{c.w, r});
    };
    auto compute = [&](const Batch& bt, int y) {
      if constexpr (ST) {
        row(cur, bt.t0, up, bt.d0, bt.l0, bt.r0);
        if (y + 1 < ye) row(bt.d0, bt.t1, cur, bt.d1, bt.l1, bt.r1);
        up = bt.d0;
        cur = bt.d1;
      } else {
        row(bt.d0, bt.t0, bt.d0, bt.d0, 0.f, 0.f);
        if (y + 1 < ye) row(bt.d1, bt.t1, bt.d1, bt.d1, 0.f, 0.f);
      }
    };
    // ping-pong buffers (no register copies, which would make every batch wait for the next)
    Batch A, Bn;
    load(A, ys);
    for (int y = ys; y < ye; y += 4) {
      // a batch past the segment's end is not loaded (ys, ye are uniform per wave: a wave's lanes
      // share their row segment, TX >= 64): at C2 a segment is ONE batch, and the two unconditional
      // prefetches were 2/3 of the loads issued
      if (y + 2 < ye) load(Bn, y + 2);
      compute(A, y);
      if (y + 4 < ye) load(A, y + 4);
      if (y + 2 < ye) compute(Bn, y + 2);
    }
  }
  // block partials: wave sums (fixed butterflies), then the 4 waves in order; explicit scalars
  // (a per-thread array here is promoted to LDS by the compiler)
  const float v0 = wave_sum(s_it[0] + s_it[1]), v1 = wave_sum(s_p[0] + s_p[1]), v2 = wave_sum(s_t[0] + s_t[1]);
  const float v3 = wave_sum((s_bce2[0] + s_bce2[1]) * kLn2), v4 = wave_sum(s_rd[0] + s_rd[1]);
  const float v5 = wave_sum(0.125f * g.eps * (s_g2[0] + s_g2[1]) + (s_q2[0] + s_q2[1]) / g.eps);
  __shared__ float fr[4][6];
  __shared__ int ir[4][3];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) {  // c_*: already whole-wave counts (ballots)
    fr[wave][0] = v0;
    fr[wave][1] = v1;
    fr[wave][2] = v2;
    fr[wave][3] = v3;
    fr[wave][4] = v4;
    fr[wave][5] = v5;
    ir[wave][0] = c_i;
    ir[wave][1] = c_p;
    ir[wave][2] = c_t;
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

// The fixed-order reduction of the row kernel's partials: a one-block launch (the launch boundary
// is the hand-off; folding it into the forward's last block was measured slower both ways: a
// same-address agent-scope ticket serialises ~2048 atomics, +20 us at C2; per-block flags polled
// by the grid's last block, +4-7 us). Every load is issued before any arithmetic (one memory round
// trip): the float partials straight into registers (thread k owns blocks k, k + 256, ...; summed
// in double in that order, fixed butterflies), the per-block counters staged in LDS and summed per
// sample by G lanes. Deterministic.
constexpr int LOSS_MAX_BLOCKS = 2048;

__device__ __forceinline__ void store_counts(const LossRowArgs& a, int b, int ci, int cp, int ct) {
  if (a.counts) {
    a.counts[b * 3 + 0] = ci;
    a.counts[b * 3 + 1] = cp;
    a.counts[b * 3 + 2] = ct;
  }
  if (a.scores) {  // fp32 arithmetic exactly as the reference metric (src/metrics.py:67-70, evaluate.py:91-94)
    const float fi = (float)ci, fp = (float)cp, ft = (float)ct, sm = a.g.smooth;
    a.scores[b * 2 + 0] = (2.f * fi + sm) / (fp + ft + sm);
    a.scores[b * 2 + 1] = (fi + sm) / (fp + ft - fi + sm);
  }
}

__device__ void finalize_rows_store(const LossArgs& g, const double* tot, float* terms);

__global__ __launch_bounds__(256) void loss_finalize_rows_kernel(LossRowArgs a) {
  const LossArgs& g = a.g;
  const int nblk = g.B * a.bands, tid = threadIdx.x;
  constexpr int PB = LOSS_MAX_BLOCKS / 256, PI = LOSS_MAX_BLOCKS * 3 / 256;
  __shared__ double red[4][6];
  __shared__ int si[LOSS_MAX_BLOCKS * 3];
  float v[PB][6];
  int vi[PI];
#pragma unroll
  for (int i = 0; i < PB; ++i) {
    const int k = tid + 256 * i;
#pragma unroll
    for (int j = 0; j < 6; ++j) v[i][j] = k < nblk ? g.fpart[k * 6 + j] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < PI; ++i) {
    const int k = tid + 256 * i;
    vi[i] = k < nblk * 3 ? g.ipart[k] : 0;
  }
#pragma unroll
  for (int i = 0; i < PI; ++i) si[tid + 256 * i] = vi[i];
  double s[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    s[j] = 0.0;
#pragma unroll
    for (int i = 0; i < PB; ++i) s[j] += (double)v[i][j];
    s[j] = wave_sum_d(s[j]);
  }
  const int lane = tid & 63, wave = tid >> 6;
  if (lane == 0)
#pragma unroll
    for (int j = 0; j < 6; ++j) red[wave][j] = s[j];
  __syncthreads();
  {  // G lanes (a power of two <= 64) per sample, uniform trip count so the butterflies run with
     // every lane active
    const int bps = a.bands;
    int G = 1;
    while (G < 64 && g.B * G * 2 <= 256) G *= 2;
    const int grp = tid / G, gl = tid % G, ngrp = 256 / G;
    const int iters = (g.B + ngrp - 1) / ngrp;
    for (int it = 0; it < iters; ++it) {
      const int b = grp + it * ngrp;
      int ci = 0, cp = 0, ct = 0;
      if (b < g.B)
        for (int k = gl; k < bps; k += G) {
          const int blk = b * bps + k;
          ci += si[blk * 3 + 0];
          cp += si[blk * 3 + 1];
          ct += si[blk * 3 + 2];
        }
      for (int off = 1; off < G; off <<= 1) {
        ci += __shfl_xor(ci, off, 64);
        cp += __shfl_xor(cp, off, 64);
        ct += __shfl_xor(ct, off, 64);
      }
      if (gl == 0 && b < g.B) store_counts(a, b, ci, cp, ct);
    }
  }
  if (tid == 0) {
    double tot[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) tot[j] = ((red[0][j] + red[1][j]) + red[2][j]) + red[3][j];
    finalize_rows_store(g, tot, a.terms);
  }
}

__device__ void finalize_rows_store(const LossArgs& g, const double* tot, float* terms) {
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


// rows per block of the whole-row forward
// about 4 blocks per CU: enough row batches per thread that the waves of a SIMD drift out of
// phase (loads of one overlapping arithmetic of another); 2048 blocks (2 batches) measured 15 %
// slower at B = 64
constexpr int LOSS_TARGET_BLOCKS = 1024;
static int loss_rows(int B, int H, int W) {
  // a multiple of RY x LOSS_ROW_BATCH rows (RY row segments per block) so no thread pads its last
  // batch; at least as many rows as keep the block count near the target
  const int ry = 256 / std::min(std::max(W / 4, 1), 256), q = ry * LOSS_ROW_BATCH;
  // at least 4 row batches per thread: small problems (C2: 16.8 MB) get fewer, fuller blocks —
  // 256 instead of 1024 at C2, 21.5 -> 18.0 us cold (profiles/r3_q21_loss_rowmul.txt); the
  // bandwidth regime (B = 64) keeps ~1024
  int r = (int)std::max<int64_t>(4 * q, cdiv((int64_t)B * H, LOSS_TARGET_BLOCKS));
  r = (int)cdiv(r, q) * q * std::max(1, tune_get(PIS_TUNE_LOSS_ROWMUL));
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
// Head forward fused with the loss forward (SURVEY §7 hard part 6): the U-Net's
// 1x1 output conv + sigmoid (src/unet.py:206-210) and every Stage-II loss term with the per-sample
// counters (src/loss.py:130-160, src/pde.py:124-212, src/metrics.py:57-71) in ONE pass over the
// 64-channel head input. A block owns R whole image rows of one sample:
//  1. u of image rows y0-1 .. y0+R (reflect-resolved; the two halo rows recomputed from their own
//     256 B/px, which the neighbouring bands fetch too: L2 / Infinity-Cache hits) into LDS, 16 lanes
//     per pixel exactly as head_fwd64_kernel (same fma order and DPP row sum, so z and u are bitwise
//     those of pis_head_fwd); the interior rows' z and u are written out (the model's outputs);
//  2. the loss partials of its R rows from LDS (u and its reflect neighbours) and the targets, as
//     loss_fwd_kernel; one finalize launch (loss_finalize_rows_kernel) reduces the [B][bands]
//     partials in fixed order.
// HBM per pixel: 256 B of x + 4 B of t read, 8 B of z, u written. The loss's own p / t pass (8 B/px,
// latency-bound at C2) and its launch are gone from the step.
// ---------------------------------------------------------------------------
struct HeadLossFwdArgs {
  const float* x;
  int ldx;
  const float* w;
  const float* bias;
  float* z;
  float* u;
  int R;          // image rows per block
  LossRowArgs a;  // the loss part: a.g (t, B, H, W, weights, partials), a.rows = R, a.bands, outputs
};

// NT threads per block (NG = NT / 16 pixel groups): 1024 at W % 512 == 0 (C2: 256 blocks of 16
// waves, four waves per SIMD to cover the HBM latency; one staged row per chunk), else 256
// D3 (pis_tune key 38 = 2): three register sets, so two chunks' loads are in flight while one is summed
template <bool RD, bool PF, int PP, int NT = 256, bool D3 = false>
__global__ __launch_bounds__(NT) void head_loss_fwd_kernel(HeadLossFwdArgs h) {
  constexpr int NG = NT / 16, NWV = NT / 64;
  constexpr bool ST = RD || PF;
  extern __shared__ __attribute__((aligned(16))) float su[];  // [R + 2][SW]: image column c at c + 4
  const LossArgs& g = h.a.g;
  const int H = g.H, W = g.W, SW = W + 8;
  // XCD-grouped (consecutive bands of a sample on one XCD, xcd_remap2) and alternating walk
  // direction (even bands bottom-up, odd bands top-down): the two blocks on either side of a band
  // boundary fetch its two rows at the same time — both at their start, or both at their end — so
  // the second fetch of a halo row is an L2 hit instead of an HBM read
  const Remap2 rmp = xcd_remap2();
  const int band = rmp.bid, b = rmp.batch;
  const int y0 = band * h.R, nr = min(h.R, H - y0);
  const bool rev = (band & 1) == 0;
  const int tid = threadIdx.x, sub = tid & 15, grp = tid >> 4;
  const size_t HW = (size_t)H * W;
  const float* xb = h.x + (size_t)b * HW * h.ldx + 4 * sub;
  const f32x4 wv = *reinterpret_cast<const f32x4*>(h.w + 4 * sub);
  const float bias = h.bias[0];
  // the loss pass's first target item of this thread (row 1 + ry, column item q), loaded now so
  // its HBM latency hides under the head pass instead of following the barrier (at C2 every
  // thread has exactly this one item)
  const int W4 = W >> 2, TX = min(W4, NT), RY = NT / TX;
  const int q = tid % TX, ry = tid / TX;
  const float* tt = h.a.g.t + (size_t)b * HW;
  const bool tpre_ok = ry < RY && q < W4 && 1 + ry <= nr;
  f32x4 tpre = {0.f, 0.f, 0.f, 0.f};
  if (tpre_ok) tpre = *reinterpret_cast<const f32x4*>(tt + (size_t)(y0 + ry) * W + 4 * q);
  // 1. u of the staged rows: a chunk is NG PP consecutive pixels of one staged row (W % (NG PP) == 0),
  // PP per 16-lane group; two register sets, so the next chunk's loads are in flight while this
  // one's sums run
  const int cpr = W / (NG * PP), nchunk = (nr + 2) * cpr;
  f32x4 xa[PP], xn[PP];
  auto srow = [&](int ch) { const int r = ch / cpr; return rev ? nr + 1 - r : r; };  // staged row of chunk ch
  auto load = [&](f32x4 (&xv)[PP], int ch) __attribute__((always_inline)) {
    const int r = srow(ch), x0 = (ch - (ch / cpr) * cpr) * (NG * PP) + grp;  // block-uniform r
    const int gy = clampi(refl(y0 - 1 + r, H), 0, H - 1);
    const float* row = xb + (size_t)gy * W * h.ldx;
#pragma unroll
    for (int j = 0; j < PP; ++j) xv[j] = *reinterpret_cast<const f32x4*>(row + (size_t)(x0 + NG * j) * h.ldx);
  };
  auto head = [&](const f32x4 (&xv)[PP], int ch) __attribute__((always_inline)) {
    const int r = srow(ch), x0 = (ch - (ch / cpr) * cpr) * (NG * PP) + grp;
    const bool interior = r >= 1 && r <= nr;
    const size_t orow = (size_t)b * HW + (size_t)(y0 - 1 + r) * W;
#pragma unroll
    for (int j = 0; j < PP; ++j) {
      float s = 0.f;
      s = fmaf(xv[j][0], wv[0], s);
      s = fmaf(xv[j][1], wv[1], s);
      s = fmaf(xv[j][2], wv[2], s);
      s = fmaf(xv[j][3], wv[3], s);
      s = group16_sum(s);  // as head_fwd64_kernel (csrc/pointwise.hip): z bitwise pis_head_fwd's
      if (sub == 0) {
        const int xx = x0 + NG * j;
        const float zz = s + bias;
        const float uu = 1.f / (1.f + expf(-zz));
        su[r * SW + 4 + xx] = uu;
        if (interior) {
          h.z[orow + xx] = zz;
          h.u[orow + xx] = uu;
        }
      }
    }
  };
  if constexpr (D3) {
    f32x4 xc[PP];
    if (nchunk > 0) load(xa, 0);
    if (nchunk > 1) load(xn, 1);
    for (int ch = 0; ch < nchunk; ch += 3) {  // a ring of three register sets (no copies)
      if (ch + 2 < nchunk) load(xc, ch + 2);
      head(xa, ch);
      if (ch + 3 < nchunk) load(xa, ch + 3);
      if (ch + 1 < nchunk) head(xn, ch + 1);
      if (ch + 4 < nchunk) load(xn, ch + 4);
      if (ch + 2 < nchunk) head(xc, ch + 2);
    }
  } else {
    if (nchunk > 0) load(xa, 0);
    for (int ch = 0; ch < nchunk; ch += 2) {  // ping-pong register sets (no copies)
      if (ch + 1 < nchunk) load(xn, ch + 1);
      head(xa, ch);
      if (ch + 2 < nchunk) load(xa, ch + 2);
      if (ch + 1 < nchunk) head(xn, ch + 1);
    }
  }
  // loss pass: TX threads per row, RY rows per pass; item = 4 pixels
  __syncthreads();
  if (ST) {  // reflect halo columns: column -1 is column 1, column W is column W-2
    for (int r = tid; r < nr + 2; r += NT) {
      su[r * SW + 3] = su[r * SW + 5];
      su[r * SW + 4 + W] = su[r * SW + 2 + W];
    }
    __syncthreads();
  }
  // 2. the loss partials of rows y0 .. y0 + nr - 1 (staged rows 1 .. nr), as loss_fwd_kernel
  constexpr float kLn2 = 0.69314718055994531f, kClamp2 = -144.26950408889634f;  // -100 / ln 2
  float s_it = 0.f, s_p = 0.f, s_t = 0.f, s_bce2 = 0.f, s_rd = 0.f, s_g2 = 0.f, s_q2 = 0.f;
  int c_i = 0, c_p = 0, c_t = 0;
  // W4 > NT (W > 4 NT, e.g. W = 1280 at 256 threads): a thread walks every TX-th item of its rows
  for (int xq = q; ry < RY && xq < W4; xq += TX) {
    for (int r = 1 + ry; r <= nr; r += RY) {
      const f32x4 tv = (xq == q && r == 1 + ry) ? tpre  // prefetched at the kernel's start
                                                : *reinterpret_cast<const f32x4*>(tt + (size_t)(y0 - 1 + r) * W + 4 * xq);
      const float* sc = su + r * SW + 4 + 4 * xq;
      const f32x4 pv = *reinterpret_cast<const f32x4*>(sc);
      f32x4 uv = pv, dv = pv;
      float lft = 0.f, rgt = 0.f;
      if (ST) {
        uv = *reinterpret_cast<const f32x4*>(sc - SW);
        dv = *reinterpret_cast<const f32x4*>(sc + SW);
        lft = sc[-1];
        rgt = sc[4];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
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
        if (ST) {
          const float ul = i == 0 ? lft : pv[i - 1], ur = i == 3 ? rgt : pv[i + 1];
          const float uu = uv[i], ud = dv[i];
          const float qq = fmaf(-p, p, p);  // p (1 - p)
          if (RD) {
            const float lap = (uu + ud) + (ul + ur) - 4.f * p;
            const float rr = fmaf(g.D, lap, g.rx * qq * (p - g.a));
            s_rd = fmaf(rr, rr, s_rd);
          }
          if (PF) {
            const float gx = ur - ul, gy2 = ud - uu;  // 2x the central differences
            s_g2 = fmaf(gx, gx, fmaf(gy2, gy2, s_g2));
            s_q2 = fmaf(qq, qq, s_q2);
          }
        }
      }
    }
  }
  const float v0 = wave_sum(s_it), v1 = wave_sum(s_p), v2 = wave_sum(s_t), v3 = wave_sum(s_bce2 * kLn2);
  const float v4 = wave_sum(s_rd), v5 = wave_sum(0.125f * g.eps * s_g2 + s_q2 / g.eps);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    c_i += __shfl_xor(c_i, off, 64);
    c_p += __shfl_xor(c_p, off, 64);
    c_t += __shfl_xor(c_t, off, 64);
  }
  __syncthreads();  // su is dead: its first words take the wave partials
  float* fr = su;                                    // [NWV][6]
  int* ir = reinterpret_cast<int*>(su + 6 * NWV);    // [NWV][3]
  const int lane = tid & 63, wave = tid >> 6;
  if (lane == 0) {
    fr[wave * 6 + 0] = v0;
    fr[wave * 6 + 1] = v1;
    fr[wave * 6 + 2] = v2;
    fr[wave * 6 + 3] = v3;
    fr[wave * 6 + 4] = v4;
    fr[wave * 6 + 5] = v5;
    ir[wave * 3 + 0] = c_i;
    ir[wave * 3 + 1] = c_p;
    ir[wave * 3 + 2] = c_t;
  }
  __syncthreads();
  const int blk = b * h.a.bands + band;
  if (tid < 6) {  // the waves in fixed order
    float v = fr[tid];
#pragma unroll
    for (int w = 1; w < NWV; ++w) v += fr[6 * w + tid];
    g.fpart[blk * 6 + tid] = v;
  } else if (tid < 9) {
    const int j = tid - 6;
    int c = ir[j];
#pragma unroll
    for (int w = 1; w < NWV; ++w) c += ir[3 * w + j];
    g.ipart[blk * 3 + j] = c;
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
    auto one = [&](int k, const f32x4& xv) __attribute__((always_inline)) {
      const float d = sdz[k];
      if (c4 == 0) accb += d;
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o[j] = xv[j] > 0.f ? d * wv[j] : 0.f;
        acc[j] = fmaf(d, xv[j], acc[j]);
      }
      *reinterpret_cast<f32x4*>(g.dx + (p0 + k) * g.lddx + 4 * c4) = o;
    };
    // four pixels' head-input loads issued together (a quarter of the round trips per thread;
    // the partial sums take the pixels in the same order as one at a time)
    const int n = nr * W;
    int k = pr;
    for (; k + 3 * rows < n; k += 4 * rows) {
      f32x4 xv[4];
#pragma unroll
      for (int u4 = 0; u4 < 4; ++u4) xv[u4] = *reinterpret_cast<const f32x4*>(g.x + (p0 + k + u4 * rows) * g.ldx + 4 * c4);
#pragma unroll
      for (int u4 = 0; u4 < 4; ++u4) one(k + u4 * rows, xv[u4]);
    }
    for (; k < n; k += rows) one(k, *reinterpret_cast<const f32x4*>(g.x + (p0 + k) * g.ldx + 4 * c4));
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

// workspace: [16 B reserved][fpart: nblk x 6 floats][ipart: nblk x 3 ints], nblk = the larger of
// the two plans; no state is carried between calls
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
    if (rd && pf) hipLaunchKernelGGL((loss_fwd_rows_kernel<true, true>), grid, dim3(256), 0, s, a);
    else if (rd) hipLaunchKernelGGL((loss_fwd_rows_kernel<true, false>), grid, dim3(256), 0, s, a);
    else if (pf) hipLaunchKernelGGL((loss_fwd_rows_kernel<false, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((loss_fwd_rows_kernel<false, false>), grid, dim3(256), 0, s, a);
    const int rc = launch_status("loss_fwd_rows");
    if (rc) return rc;
    hipLaunchKernelGGL(loss_finalize_rows_kernel, dim3(1), dim3(256), 0, s, a);
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

// rows per block of the fused head + loss forward: 4096 / W, i.e. 4096 pixels (8 at W = 512: 512
// blocks of 10 staged rows at C2, two per CU; 4 at W = 1024), doubled while the batch's row bands
// exceed LOSS_MAX_BLOCKS; pis_tune key 36 overrides. At C2 8 rows ran the kernel in 131 us against
// 134-145 us at 16 and 144 at 4 (0.54 vs 0.48-0.52 of 8 TB/s live; profiles/r4_ah_head_loss_rows.txt)
// although a quarter of the head input is fetched twice (the halo rows, mostly from L2)
static int head_loss_fwd_rows(int B, int H, int W) {
  const int t = tune_get(PIS_TUNE_HEAD_LOSS_ROWS);
  int r = t > 0 ? t : std::max(2, std::min(16, 4096 / std::max(1, W)));
  if (t <= 0)
    while (r < H && (int64_t)B * ((H + r - 1) / r) > LOSS_MAX_BLOCKS) r *= 2;
  return std::max(1, std::min(r, H));
}

// pixels per 16-lane group in flight in the fused head + loss forward (W % (NG PP) == 0), 0: none fits;
// W % 512 == 0 runs 1024-thread blocks (64 groups x 8 pixels: one 512-pixel row per chunk)
static int head_loss_fwd_pp(int W) { return W % 256 == 0 ? 16 : W % 128 == 0 ? 8 : W % 64 == 0 ? 4 : 0; }
static bool head_loss_fwd_wide(int W) { return W % 512 == 0 && tune_get(PIS_TUNE_HEAD_LOSS_WIDE) != 0; }

extern "C" size_t pis_head_loss_fwd_ws(int B, int H, int W) {
  // sized for one row per block, so a later key-36 change cannot outgrow a planned workspace
  const size_t nblk = (size_t)B * H;
  (void)W;
  return 16 + nblk * (6 * sizeof(float) + 3 * sizeof(int)) + 256;
}

// the staged u rows, (R + 2) x (W + 8) floats, must fit one workgroup's LDS (160 KB on gfx950); a
// shape that does not (e.g. B = 128 at 1024^2: R = 64, 272 KB) takes pis_head_fwd + pis_loss_fwd
static constexpr size_t kHeadLossFwdMaxLds = 160 * 1024;
static size_t head_loss_fwd_smem(int R, int W) { return (size_t)(R + 2) * (W + 8) * sizeof(float); }

extern "C" int pis_head_loss_fwd_ok(int B, int H, int W, int C) {
  const int R = head_loss_fwd_rows(B, H, W);
  return C == 64 && B > 0 && H >= 2 && W >= 8 && W <= 2048 && head_loss_fwd_pp(W) > 0 &&
         (int64_t)B * ((H + R - 1) / R) <= LOSS_MAX_BLOCKS && head_loss_fwd_smem(R, W) <= kHeadLossFwdMaxLds;
}

extern "C" int pis_head_loss_fwd(const float* x, int ldx, const float* w, const float* bias, const float* t,
                                 float* z, float* u, int B, int H, int W, int C, const pis_loss_params* prm,
                                 float* out_terms, int* counts, float* scores, void* ws, size_t ws_bytes,
                                 pis_stream_t stream) {
  PIS_CHECK_ARG(x && w && bias && t && z && u && prm && out_terms, "pis_head_loss_fwd: bad arguments");
  PIS_CHECK_ARG(pis_head_loss_fwd_ok(B, H, W, C),
                "pis_head_loss_fwd: needs C == 64, W % 64 == 0, W <= 2048, H >= 2, at most 2048 row bands "
                "and staged rows within 160 KB of LDS (use pis_head_fwd + pis_loss_fwd)");
  PIS_CHECK_ARG(ldx % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)t & 15) == 0 && ((uintptr_t)w & 15) == 0,
                "pis_head_loss_fwd: x, w, t must be 16-byte aligned with ldx % 4 == 0");
  PIS_CHECK_ARG(ws && ws_bytes >= pis_head_loss_fwd_ws(B, H, W), "pis_head_loss_fwd: workspace too small");
  HeadLossFwdArgs h{};
  h.x = x; h.ldx = ldx; h.w = w; h.bias = bias; h.z = z; h.u = u;
  h.R = head_loss_fwd_rows(B, H, W);
  LossArgs& g = h.a.g;
  g.p = u; g.t = t; g.B = B; g.H = H; g.W = W;
  g.dice_w = prm->dice_w; g.bce_w = prm->bce_w; g.rd_w = prm->rd_w; g.pf_w = prm->pf_w;
  g.smooth = prm->smooth; g.D = prm->D; g.a = prm->a; g.eps = prm->eps;
  g.rx = (prm->flags & PIS_LOSS_NO_REACTION) ? 0.f : 1.f; g.thr = prm->thr;
  const int bands = (H + h.R - 1) / h.R;
  const int64_t nblk = (int64_t)B * bands;
  g.fpart = (float*)((char*)ws + 16);
  g.ipart = (int*)((char*)ws + 16 + (size_t)nblk * 6 * sizeof(float));
  h.a.rows = h.R;
  h.a.bands = bands;
  h.a.terms = out_terms; h.a.counts = counts; h.a.scores = scores;
  const bool all = prm->flags & PIS_LOSS_ALL_TERMS;
  const bool rd = all || prm->rd_w > 0.f, pf = all || prm->pf_w > 0.f;
  const int pp = head_loss_fwd_pp(W);
  const bool wide = head_loss_fwd_wide(W);
  const bool wide3 = wide && tune_get(PIS_TUNE_HEAD_LOSS_WIDE) == 2;
  const size_t smem = head_loss_fwd_smem(h.R, W);
  const dim3 grid(bands, B);
  hipStream_t s = (hipStream_t)stream;
  const double nbytes = (double)B * H * W * (4.0 * C + 12.0);
  launch_hook("head_loss_fwd", 0, s, nbytes);
#define PIS_HLF(RDV, PFV)                                                                                         \
  do {                                                                                                            \
    if (wide && wide3) hipLaunchKernelGGL((head_loss_fwd_kernel<RDV, PFV, 8, 1024, true>), grid, dim3(1024), smem, s, h); \
    else if (wide) hipLaunchKernelGGL((head_loss_fwd_kernel<RDV, PFV, 8, 1024>), grid, dim3(1024), smem, s, h);   \
    else if (pp == 16) hipLaunchKernelGGL((head_loss_fwd_kernel<RDV, PFV, 16>), grid, dim3(256), smem, s, h);     \
    else if (pp == 8) hipLaunchKernelGGL((head_loss_fwd_kernel<RDV, PFV, 8>), grid, dim3(256), smem, s, h);       \
    else hipLaunchKernelGGL((head_loss_fwd_kernel<RDV, PFV, 4>), grid, dim3(256), smem, s, h);                    \
  } while (0)
  if (rd && pf) PIS_HLF(true, true);
  else if (rd) PIS_HLF(true, false);
  else if (pf) PIS_HLF(false, true);
  else PIS_HLF(false, false);
#undef PIS_HLF
  launch_hook("head_loss_fwd", 1, s, nbytes);
  int rc = launch_status("head_loss_fwd");
  if (rc) return rc;
  hipLaunchKernelGGL(loss_finalize_rows_kernel, dim3(1), dim3(256), 0, s, h.a);
  return launch_status("loss_finalize");
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
  // dw and db in one launch (fixed-order sums, deterministic)
  if (!rc) rc = reduce_slabs2(g.part, (int)(grid.x * grid.y), C, dw, db ? g.part_b : nullptr, (int)(grid.x * grid.y), 1,
                              db, acc, s);
  return rc;
}
