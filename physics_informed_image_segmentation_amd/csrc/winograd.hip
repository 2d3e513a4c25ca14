// Winograd 3x3 convolutions (fwd, and dgrad on flipped weights) and weight gradients.
//
// Contents, in file order:
//   * F(2x2,3x3) / F(3x3,2x2): transforms for grids not divisible by 4 (pis_tune(11, 0));
//   * F(4x4,3x3) / F(3x3,4x4) (the default): filter, input, output, dz and merged-dz (dz2)
//     transforms — bandwidth-bound streams, one thread per tile x 4 channels, compile-time
//     Cook-Toom coefficients on the points {0, 1, -1, 1/2, -2, inf};
//   * the opt-in fully fused F(4x4) kernel (pis_tune(12, 2));
//   * the 36 batched NT GEMMs M_xi = V_xi U_xi^T: fp32 MFMA (gemm_nt_kernel) and fp32-accurate
//     bf16x6 on bf16 MFMA (gemm_nt_x6_kernel; gemm_nt_x6_bk32_kernel, the default);
//   * the fused 64->64 contraction + output transform (wino4_gemm_out_x6_kernel);
//   * launchers (launch_wino3x3 ...) and the pis_debug_gemm_nt tooling entry.
//
// With U = G g G^T (weights), V = B^T d B (input patch) and M_xi = sum_c V_xi[tile][c] U_xi[n][c],
// the outputs are Y = A^T M A: (m + 2)^2 / m^2 multiply-adds per output instead of 9.
// Workspace (floats): U[nxi][N][C], V[nxi][T][C], M[nxi][T][N], T = B (H/m) (W/m) tiles.
//
// F(2x2,3x3) matrices:
//   B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1]
//   G   = [1 0 0; 1/2 1/2 1/2; 1/2 -1/2 1/2; 0 0 1]
//   A^T = [1 1 1 0; 0 1 -1 -1]
#include "igemm.h"

namespace pis {

// U[xi][n][c] = (G g G^T)[xi] for g = w[n][tap][c] (KRSC, ldw = 9*C)
__global__ __launch_bounds__(256) void wino_filter_kernel(const float* __restrict__ w, int ldw, int N, int C,
                                                          float* __restrict__ U) {
  const int64_t NC = (int64_t)N * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < NC; e += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(e / C), c = (int)(e - (int64_t)n * C);
    float g[3][3];
#pragma unroll
    for (int t = 0; t < 9; ++t) g[t / 3][t % 3] = w[(size_t)n * ldw + t * C + c];
    float gg[4][3];  // G g
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      gg[0][s] = g[0][s];
      gg[1][s] = 0.5f * (g[0][s] + g[1][s] + g[2][s]);
      gg[2][s] = 0.5f * (g[0][s] - g[1][s] + g[2][s]);
      gg[3][s] = g[2][s];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float u0 = gg[i][0], u1 = 0.5f * (gg[i][0] + gg[i][1] + gg[i][2]);
      const float u2 = 0.5f * (gg[i][0] - gg[i][1] + gg[i][2]), u3 = gg[i][2];
      U[(size_t)(i * 4 + 0) * NC + e] = u0;
      U[(size_t)(i * 4 + 1) * NC + e] = u1;
      U[(size_t)(i * 4 + 2) * NC + e] = u2;
      U[(size_t)(i * 4 + 3) * NC + e] = u3;
    }
  }
}

// V[xi][t][c] = (B^T d B)[xi], d = the 4x4 input patch at rows 2ty-1.., cols 2tx-1.. (zero padded)
__global__ __launch_bounds__(256) void wino_input_kernel(const float* __restrict__ x, int ldx, int B, int H, int W,
                                                         int C, float* __restrict__ V) {
  const int c4n = C / 4, TW = W / 2, TH = H / 2;
  const int64_t T = (int64_t)B * TH * TW, TC = T * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < T * c4n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = e / c4n;
    const int c = (int)(e - t * c4n) * 4;
    const int b = (int)(t / (TH * TW)), rem = (int)(t - (int64_t)b * TH * TW);
    const int ty = rem / TW, tx = rem - ty * TW;
    f32x4 d[4][4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int h = 2 * ty - 1 + r;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int ww = 2 * tx - 1 + s;
        d[r][s] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (h >= 0 && h < H && ww >= 0 && ww < W)
          d[r][s] = *reinterpret_cast<const f32x4*>(x + (((size_t)b * H + h) * W + ww) * ldx + c);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f32x4 tr[4];  // row i of B^T d
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        tr[s] = i == 0 ? d[0][s] - d[2][s] : i == 1 ? d[1][s] + d[2][s] : i == 2 ? d[2][s] - d[1][s] : d[1][s] - d[3][s];
      }
      const f32x4 v0 = tr[0] - tr[2], v1 = tr[1] + tr[2], v2 = tr[2] - tr[1], v3 = tr[1] - tr[3];
      float* out = V + (size_t)(i * 4) * TC + t * C + c;
      *reinterpret_cast<f32x4*>(out) = v0;
      *reinterpret_cast<f32x4*>(out + TC) = v1;
      *reinterpret_cast<f32x4*>(out + 2 * TC) = v2;
      *reinterpret_cast<f32x4*>(out + 3 * TC) = v3;
    }
  }
}

template <int VW>
using fvec = float __attribute__((ext_vector_type(VW)));  // VW consecutive NHWC channels

// conv epilogue on VW channels of one output pixel (v = conv + bias): ReLU, ReLU-backward
// mask, dropout keep-scale, accumulate — the direct kernels' epilogue (igemm.hip)
template <int VW = 4>
__device__ __forceinline__ fvec<VW> conv_epilogue4(const IGemmArgs& g, size_t pix, int n, fvec<VW> v,
                                                   fvec<VW> sc4) {
  if (g.flags & PIS_RELU) {
#pragma unroll
    for (int k = 0; k < VW; ++k) v[k] = fmaxf(v[k], 0.f);
  }
  if (g.flags & PIS_MASK) {
    const fvec<VW> mk = *reinterpret_cast<const fvec<VW>*>(g.mask + pix * g.ldm + n);
#pragma unroll
    for (int k = 0; k < VW; ++k) v[k] = mk[k] > 0.f ? v[k] : 0.f;
  }
  v *= sc4;
  float* dst = g.dst + pix * g.ldd + n;
  if (g.flags & PIS_ACCUMULATE) v += *reinterpret_cast<const fvec<VW>*>(dst);
  *reinterpret_cast<fvec<VW>*>(dst) = v;
  return v;
}

// the same with the ReLU-backward mask already loaded (mk; ignored without PIS_MASK)
__device__ __forceinline__ f32x4 conv_epilogue4m(const IGemmArgs& g, size_t pix, int n, f32x4 v, f32x4 sc4, f32x4 mk) {
  if (g.flags & PIS_RELU) {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = fmaxf(v[k], 0.f);
  }
  if (g.flags & PIS_MASK) {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = mk[k] > 0.f ? v[k] : 0.f;
  }
  v *= sc4;
  float* dst = g.dst + pix * g.ldd + n;
  if (g.flags & PIS_ACCUMULATE) v += *reinterpret_cast<const f32x4*>(dst);
  *reinterpret_cast<f32x4*>(dst) = v;
  return v;
}

// VW channels with the mask already loaded (mk; ignored without PIS_MASK)
template <int VW>
__device__ __forceinline__ fvec<VW> conv_epilogue_vm(const IGemmArgs& g, size_t pix, int n, fvec<VW> v, fvec<VW> sc4,
                                                     fvec<VW> mk) {
  if (g.flags & PIS_RELU) {
#pragma unroll
    for (int k = 0; k < VW; ++k) v[k] = fmaxf(v[k], 0.f);
  }
  if (g.flags & PIS_MASK) {
#pragma unroll
    for (int k = 0; k < VW; ++k) v[k] = mk[k] > 0.f ? v[k] : 0.f;
  }
  v *= sc4;
  float* dst = g.dst + pix * g.ldd + n;
  if (g.flags & PIS_ACCUMULATE) v += *reinterpret_cast<const fvec<VW>*>(dst);
  *reinterpret_cast<fvec<VW>*>(dst) = v;
  return v;
}

template <int VW = 4>
__device__ __forceinline__ fvec<VW> max4(fvec<VW> a, fvec<VW> b, fvec<VW> c, fvec<VW> d) {
  fvec<VW> m;
#pragma unroll
  for (int k = 0; k < VW; ++k) m[k] = fmaxf(fmaxf(a[k], b[k]), fmaxf(c[k], d[k]));
  return m;
}

// Y = A^T M A per tile and 4 output channels, then the conv epilogue of the direct
// kernels (bias, ReLU, ReLU-backward mask, dropout keep-scale, accumulate).
__global__ __launch_bounds__(256) void wino_output_kernel(const float* __restrict__ Mt, IGemmArgs g, int B) {
  const int N = g.N, n4n = N / 4, TW = g.W / 2, TH = g.H / 2;
  const int64_t T = (int64_t)B * TH * TW, TN = T * N;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < T * n4n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = e / n4n;
    const int n = (int)(e - t * n4n) * 4;
    const int b = (int)(t / (TH * TW)), rem = (int)(t - (int64_t)b * TH * TW);
    const int ty = rem / TW, tx = rem - ty * TW;
    f32x4 m[4][4];
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) m[xi / 4][xi % 4] = *reinterpret_cast<const f32x4*>(Mt + xi * TN + t * N + n);
    f32x4 tr[2][4];  // A^T M
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      tr[0][s] = m[0][s] + m[1][s] + m[2][s];
      tr[1][s] = m[1][s] - m[2][s] - m[3][s];
    }
    f32x4 bias4 = {0.f, 0.f, 0.f, 0.f}, sc4 = {1.f, 1.f, 1.f, 1.f};
    if (g.bias) bias4 = *reinterpret_cast<const f32x4*>(g.bias + n);
    if (g.flags & PIS_SCALE) sc4 = *reinterpret_cast<const f32x4*>(g.scale + (size_t)b * N + n);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f32x4 y0 = tr[i][0] + tr[i][1] + tr[i][2];
      const f32x4 y1 = tr[i][1] - tr[i][2] - tr[i][3];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const size_t pix = ((size_t)b * g.H + 2 * ty + i) * g.W + 2 * tx + j;
        conv_epilogue4(g, pix, n, (j == 0 ? y0 : y1) + bias4, sc4);
      }
    }
  }
}

// ---- weight gradient: the dual algorithm F(3x3, 2x2) -------------------------------
// dW[r][s] = sum_tiles G^T (E (.) V) G per (n, c), with V = B^T d B (the forward's input
// transform) and E = A e A^T from the 2x2 output-gradient tile e; the 16 contractions over
// tiles run on the split-K MFMA weight-gradient GEMM (wgrad.hip).
//   A = [1 0; 1 1; 1 -1; 0 -1],  G^T = [1 1/2 1/2 0; 0 1/2 -1/2 0; 0 1/2 1/2 1]

// E[xi][t][n] = (A e A^T)[xi], e = dz at output pixels (2ty + i, 2tx + j)
__global__ __launch_bounds__(256) void wino_dz_kernel(const float* __restrict__ dz, int ldz, int B, int H, int W,
                                                      int N, float* __restrict__ E) {
  const int n4n = N / 4, TW = W / 2, TH = H / 2;
  const int64_t T = (int64_t)B * TH * TW, TN = T * N;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < T * n4n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = e / n4n;
    const int n = (int)(e - t * n4n) * 4;
    const int b = (int)(t / (TH * TW)), rem = (int)(t - (int64_t)b * TH * TW);
    const int ty = rem / TW, tx = rem - ty * TW;
    f32x4 g[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        g[i][j] = *reinterpret_cast<const f32x4*>(dz + (((size_t)b * H + 2 * ty + i) * W + 2 * tx + j) * ldz + n);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f32x4 tr[2];  // row k of A e
#pragma unroll
      for (int j = 0; j < 2; ++j)
        tr[j] = k == 0 ? g[0][j] : k == 1 ? g[0][j] + g[1][j] : k == 2 ? g[0][j] - g[1][j] : -g[1][j];
      float* out = E + (size_t)(k * 4) * TN + t * N + n;
      *reinterpret_cast<f32x4*>(out) = tr[0];
      *reinterpret_cast<f32x4*>(out + TN) = tr[0] + tr[1];
      *reinterpret_cast<f32x4*>(out + 2 * TN) = tr[0] - tr[1];
      *reinterpret_cast<f32x4*>(out + 3 * TN) = -tr[1];
    }
  }
}

// dw[n][r][s][c] (+)= (G^T M G)[r][s], M[xi][n][c] the reduced tile sums
__global__ __launch_bounds__(256) void wino_wgrad_out_kernel(const float* __restrict__ M, int N, int C,
                                                             float* __restrict__ dw, int accumulate) {
  const int64_t NC = (int64_t)N * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < NC; e += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(e / C), c = (int)(e - (int64_t)n * C);
    float m[4][4];
#pragma unroll
    for (int xi = 0; xi < 16; ++xi) m[xi / 4][xi % 4] = M[xi * NC + e];
    float tr[3][4];  // G^T M
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      tr[0][l] = m[0][l] + 0.5f * (m[1][l] + m[2][l]);
      tr[1][l] = 0.5f * (m[1][l] - m[2][l]);
      tr[2][l] = 0.5f * (m[1][l] + m[2][l]) + m[3][l];
    }
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const float w0 = tr[r][0] + 0.5f * (tr[r][1] + tr[r][2]);
      const float w1 = 0.5f * (tr[r][1] - tr[r][2]);
      const float w2 = 0.5f * (tr[r][1] + tr[r][2]) + tr[r][3];
      float* o = dw + ((size_t)n * 9 + r * 3) * C + c;
      if (accumulate) {
        o[0] += w0;
        o[C] += w1;
        o[2 * C] += w2;
      } else {
        o[0] = w0;
        o[C] = w1;
        o[2 * C] = w2;
      }
    }
  }
}

// ---- F(4x4, 3x3): 6x6 input patches, 36 contractions, 2.25 MACs per output (direct: 9) ----
// Cook-Toom points {0, 1, -1, 1/2, -2, inf}: fp32 error 1.8e-6 relative (norm, 512-channel
// layers against float64) where the usual {0, +-1, +-2} gives 2.7e-6 and F(2x2,3x3) 0.4e-6.
// V = BT d BT^T, U = G g G^T, Y = AT M AT^T. Per output pixel the transformed operands are
// 36/16 = 2.25 floats per channel (F(2x2): 4), so the transforms stream less HBM too.
// The tile grid needs H % 4 == W % 4 == 0.
__host__ __device__ constexpr float w4_bt(int i, int k) {
  constexpr float m[6][6] = {{1.f, -1.5f, -2.f, 1.5f, 1.f, 0.f},  {0.f, -1.f, 0.5f, 2.5f, 1.f, 0.f},
                             {0.f, 1.f, -2.5f, 0.5f, 1.f, 0.f},   {0.f, -2.f, -1.f, 2.f, 1.f, 0.f},
                             {0.f, 0.5f, -1.f, -0.5f, 1.f, 0.f},  {0.f, 1.f, -1.5f, -2.f, 1.5f, 1.f}};
  return m[i][k];
}
__host__ __device__ constexpr float w4_g(int i, int k) {
  constexpr float m[6][3] = {{1.f, 0.f, 0.f},
                             {1.f / 3, 1.f / 3, 1.f / 3},
                             {-1.f / 3, 1.f / 3, -1.f / 3},
                             {-16.f / 15, -8.f / 15, -4.f / 15},
                             {1.f / 15, -2.f / 15, 4.f / 15},
                             {0.f, 0.f, 1.f}};
  return m[i][k];
}
__host__ __device__ constexpr float w4_at(int i, int k) {
  constexpr float m[4][6] = {{1.f, 1.f, 1.f, 1.f, 1.f, 0.f},
                             {0.f, 1.f, -1.f, 0.5f, -2.f, 0.f},
                             {0.f, 1.f, 1.f, 0.25f, 4.f, 0.f},
                             {0.f, 1.f, -1.f, 0.125f, -8.f, 1.f}};
  return m[i][k];
}
// acc += c * v with the compile-time coefficient c folded (0: nothing, +-1: add/sub)
template <typename T>
__device__ __forceinline__ void axpy_c(T& acc, float c, const T& v) {
  if (c == 0.f) return;
  if (c == 1.f) acc += v;
  else if (c == -1.f) acc -= v;
  else acc += c * v;
}

// (tile, channel-quad) item e -> tile t, first channel c, image b, tile index within the image;
// 32-bit divisions while e fits (a few instructions; 64-bit ones are a software routine)
template <int VW = 4>
__device__ __forceinline__ void tile_decode(int64_t e, int c4n, int tpi, int64_t& t, int& c, int& b, int& rem) {
  if (e <= 0x7fffffff) {
    const unsigned eu = (unsigned)e, tu = eu / (unsigned)c4n;
    c = (int)(eu - tu * (unsigned)c4n) * VW;
    t = tu;
    b = (int)(tu / (unsigned)tpi);
    rem = (int)(tu - (unsigned)b * (unsigned)tpi);
  } else {
    t = e / c4n;
    c = (int)(e - t * c4n) * VW;
    b = (int)(t / tpi);
    rem = (int)(t - (int64_t)b * tpi);
  }
}

// U[xi][n][c] = (G g G^T)[xi], xi = 6 i + j, for the filter g of pair e = n C + c
// With Up != NULL the transform is written as the bf16x6 hi/mid/lo planes Up[p][xi][n][c] instead
// (the fused GEMM + output-transform kernel reads its B fragments straight from them).
__device__ __forceinline__ void wino4_filter_item(const float (&g)[3][3], int64_t e, int n, int c, int N,
                                                  int64_t NC, float* __restrict__ U, int transposed,
                                                  __bf16* __restrict__ Up) {
  float gg[6][3];  // G g
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      gg[i][s] = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) axpy_c(gg[i][s], w4_g(i, k), g[k][s]);
    }
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      float u = 0.f;
#pragma unroll
      for (int s = 0; s < 3; ++s) axpy_c(u, w4_g(j, s), gg[i][s]);
      if (Up) {
        const __bf16 h = (__bf16)u;
        const float r = u - (float)h;
        const __bf16 m = (__bf16)r;
        const size_t o = (size_t)(i * 6 + j) * NC + e;
        Up[o] = h;
        Up[36 * NC + o] = m;
        Up[72 * NC + o] = (__bf16)(r - (float)m);
        continue;
      }
      // [xi][n][c] for the batched GEMMs; [xi][c][n] for the fused kernel's B operand
      U[(size_t)(i * 6 + j) * NC + (transposed ? (int64_t)c * N + n : e)] = u;
    }
}

// w: KRSC weights [N][9][C] (row pitch ldw), already in the operand's orientation (the forward's
// own weights, or pis_conv3x3_flip's copy for an input gradient). Block `bid` of `nblk`.
__device__ __forceinline__ void wino4_filter_range(const float* __restrict__ w, int ldw, int N, int C,
                                                   float* __restrict__ U, int transposed, __bf16* __restrict__ Up,
                                                   int bid, int nblk) {
  const int64_t NC = (int64_t)N * C;
  for (int64_t e = (int64_t)bid * blockDim.x + threadIdx.x; e < NC; e += (int64_t)nblk * blockDim.x) {
    const int n = (int)(e / C), c = (int)(e - (int64_t)n * C);
    float g[3][3];
#pragma unroll
    for (int t = 0; t < 9; ++t) g[t / 3][t % 3] = w[(size_t)n * ldw + t * C + c];
    wino4_filter_item(g, e, n, c, N, NC, U, transposed, Up);
  }
}

__global__ __launch_bounds__(256) void wino4_filter_kernel(const float* __restrict__ w, int ldw, int N, int C,
                                                           float* __restrict__ U, int transposed = 0,
                                                           __bf16* __restrict__ Up = nullptr) {
  wino4_filter_range(w, ldw, N, C, U, transposed, Up, blockIdx.x, gridDim.x);
}

// The input-gradient filter transform straight from the layer's ORIGINAL KRSC weights [C][9][N]
// (N = Cin, C = Cout; PIS_W_UNFLIPPED): g = the 180-degree-rotated, transposed filter, read in
// place instead of from a pis_conv3x3_flip copy. N % 32 == 0, C % 32 == 0; a block owns
// 32 n x 32 c; the 9 taps of that tile are read along n (128-B runs of the original [C][9][N]
// weights) into LDS and each thread then transforms (n, c) pairs with c fastest, so the 36
// output planes are written in runs along c as by wino4_filter_kernel.
__device__ __forceinline__ void wino4_filter_rot_tile(const float* __restrict__ w, int N, int C,
                                                      float* __restrict__ U, int transposed,
                                                      __bf16* __restrict__ Up, int tile) {
  __shared__ float sg[9][32][33];  // [tap][c][n], padded: the transform reads along c conflict-free
  const int nb = N / 32, n0 = 32 * (tile % nb), c0 = 32 * (tile / nb);
  const int tid = threadIdx.x, lx = tid & 31, ly = tid >> 5;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = ly + 8 * i;
      sg[t][c][lx] = w[((size_t)(c0 + c) * 9 + t) * N + n0 + lx];
    }
  __syncthreads();
  const int64_t NC = (int64_t)N * C;
#pragma unroll 1
  for (int i = 0; i < 4; ++i) {
    const int c = lx, nl = ly + 8 * i, n = n0 + nl;
    float g[3][3];
#pragma unroll
    for (int t = 0; t < 9; ++t) g[t / 3][t % 3] = sg[8 - t][c][nl];
    wino4_filter_item(g, (int64_t)n * C + c0 + c, n, c0 + c, N, NC, U, transposed, Up);
  }
}

__global__ __launch_bounds__(256) void wino4_filter_rot_kernel(const float* __restrict__ w, int N, int C,
                                                               float* __restrict__ U, int transposed,
                                                               __bf16* __restrict__ Up) {
  wino4_filter_rot_tile(w, N, C, U, transposed, Up, blockIdx.x);
}

// The fused kernel's fp16x3 filter planes (pis_tune key 22), C % 64 == 0: one wave per output
// channel n, lane c (+ 64 j). All 36 C U[xi][n][c] of the channel share ONE power-of-two scale t_n
// (from their max over xi and c; a first pass finds it, the second recomputes and writes):
// Uh[p][xi][n][c] = hi / lo fp16 of u t_n, then Us[n] = 1 / t_n after the planes. dgrad: the
// input-gradient filter straight from the original KRSC weights [C][9][N] (rotated, transposed;
// as wino4_filter_rot_tile), else w is [N][9][C] with row pitch ldw.
__device__ __forceinline__ void wino4_filter_h2_u(const float* __restrict__ w, int ldw, int N, int C, int dgrad,
                                                  int n, int c, float (&u)[36]) {
  float g[3][3];
#pragma unroll
  for (int t = 0; t < 9; ++t)
    g[t / 3][t % 3] = dgrad ? w[((size_t)c * 9 + 8 - t) * N + n] : w[(size_t)n * ldw + t * C + c];
  float gg[6][3];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      gg[i][s] = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) axpy_c(gg[i][s], w4_g(i, k), g[k][s]);
    }
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      float v = 0.f;
#pragma unroll
      for (int s = 0; s < 3; ++s) axpy_c(v, w4_g(j, s), gg[i][s]);
      u[6 * i + j] = v;
    }
}

__device__ __forceinline__ void wino4_filter_h2_wave(const float* __restrict__ w, int ldw, int N, int C, int dgrad,
                                                     __bf16* __restrict__ Up, int n) {
  const int lane = threadIdx.x & 63;
  float u[36];
  float m = 0.f;
  for (int c = lane; c < C; c += 64) {
    wino4_filter_h2_u(w, ldw, N, C, dgrad, n, c, u);
#pragma unroll
    for (int xi = 0; xi < 36; ++xi) m = fmaxf(m, fabsf(u[xi]));
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
  float sc, inv;
  h2_scale_pair(m, sc, inv);
  _Float16* Uh = reinterpret_cast<_Float16*>(Up);
  const size_t NC = (size_t)N * C;
  for (int c = lane; c < C; c += 64) {
    wino4_filter_h2_u(w, ldw, N, C, dgrad, n, c, u);
#pragma unroll
    for (int xi = 0; xi < 36; ++xi) {
      const float us = u[xi] * sc;
      const _Float16 h = (_Float16)us;
      const size_t o = xi * NC + (size_t)n * C + c;
      Uh[o] = h;
      Uh[36 * NC + o] = (_Float16)(us - (float)h);
    }
  }
  if (lane == 0) reinterpret_cast<float*>(Uh + 72 * NC)[n] = inv;
}

__global__ __launch_bounds__(256) void wino4_filter_h2_kernel(const float* __restrict__ w, int ldw, int N, int C,
                                                              int dgrad, __bf16* __restrict__ Up) {
  wino4_filter_h2_wave(w, ldw, N, C, dgrad, Up, 4 * blockIdx.x + (threadIdx.x >> 6));
}

// ---- F(6x6,3x3): 8 x 8 input tiles, 64 contractions per 36 outputs (16 / 9 products per output
// against F(4x4)'s 9 / 4: 21 % fewer GEMM FLOPs and V / M bytes on a divisible grid) -----------------
// Cook-Toom points {0, 1, -1, 2, -2, 1/2, -1/2, inf} (the same construction as the F(4x4) tables
// above). Measured fp32 error of the whole convolution against float64 (256 -> 64 channels, ReLU'd
// inputs): 5.4e-6 relative (norm), 1.5e-5 of the output scale at worst, against 1.8e-6 / 4.2e-6 for
// F(4x4) with {0, 1, -1, 1/2, -2}. Used for the forward and input gradient
// of the deep layers that run the batched GEMM both ways (wino6_layer); their weight gradients keep
// F(3x3,4x4) with their own transforms (no kept V). Ragged grids: the tile grid is ceil(H / 6) x
// ceil(W / 6), inputs past the image are zeros and outputs past it are not written.
__host__ __device__ constexpr float w6_bt(int i, int k) {
  constexpr float m[8][8] = {{-1.f, 0.f, 21.f / 4, 0.f, -21.f / 4, 0.f, 1.f, 0.f},
                             {0.f, 1.f, 1.f, -17.f / 4, -17.f / 4, 1.f, 1.f, 0.f},
                             {0.f, -1.f, 1.f, 17.f / 4, -17.f / 4, -1.f, 1.f, 0.f},
                             {0.f, 1.f / 2, 1.f / 4, -5.f / 2, -5.f / 4, 2.f, 1.f, 0.f},
                             {0.f, -1.f / 2, 1.f / 4, 5.f / 2, -5.f / 4, -2.f, 1.f, 0.f},
                             {0.f, 2.f, 4.f, -5.f / 2, -5.f, 1.f / 2, 1.f, 0.f},
                             {0.f, -2.f, 4.f, 5.f / 2, -5.f, -1.f / 2, 1.f, 0.f},
                             {0.f, -1.f, 0.f, 21.f / 4, 0.f, -21.f / 4, 0.f, 1.f}};
  return m[i][k];
}
__host__ __device__ constexpr float w6_g(int i, int k) {
  constexpr float m[8][3] = {{-1.f, 0.f, 0.f},
                             {-2.f / 9, -2.f / 9, -2.f / 9},
                             {-2.f / 9, 2.f / 9, -2.f / 9},
                             {1.f / 90, 1.f / 45, 2.f / 45},
                             {1.f / 90, -1.f / 45, 2.f / 45},
                             {32.f / 45, 16.f / 45, 8.f / 45},
                             {32.f / 45, -16.f / 45, 8.f / 45},
                             {0.f, 0.f, 1.f}};
  return m[i][k];
}
__host__ __device__ constexpr float w6_at(int i, int k) {
  constexpr float m[6][8] = {{1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 0.f},
                             {0.f, 1.f, -1.f, 2.f, -2.f, 1.f / 2, -1.f / 2, 0.f},
                             {0.f, 1.f, 1.f, 4.f, 4.f, 1.f / 4, 1.f / 4, 0.f},
                             {0.f, 1.f, -1.f, 8.f, -8.f, 1.f / 8, -1.f / 8, 0.f},
                             {0.f, 1.f, 1.f, 16.f, 16.f, 1.f / 16, 1.f / 16, 0.f},
                             {0.f, 1.f, -1.f, 32.f, -32.f, 1.f / 32, -1.f / 32, 1.f}};
  return m[i][k];
}

// U[xi][n][c] = (G g G^T)[xi], xi = 8 i + j, for the filter g of pair e = n C + c
__device__ __forceinline__ void wino6_filter_item(const float (&g)[3][3], int64_t e, int64_t NC, float* __restrict__ U) {
  float gg[8][3];  // G g
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      gg[i][s] = 0.f;
#pragma unroll
      for (int k = 0; k < 3; ++k) axpy_c(gg[i][s], w6_g(i, k), g[k][s]);
    }
  float* o = U + e;  // one pointer walked plane to plane (64 per-plane scalar offsets spill SGPRs)
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float u = 0.f;
#pragma unroll
      for (int s = 0; s < 3; ++s) axpy_c(u, w6_g(j, s), gg[i][s]);
      *o = u;
      o += NC;
    }
}

// the forward's weights w [N][9][C] (row pitch ldw), block bid of nblk
__device__ __forceinline__ void wino6_filter_range(const float* __restrict__ w, int ldw, int N, int C,
                                                   float* __restrict__ U, int bid, int nblk) {
  const int64_t NC = (int64_t)N * C;
  for (int64_t e = (int64_t)bid * blockDim.x + threadIdx.x; e < NC; e += (int64_t)nblk * blockDim.x) {
    const int n = (int)(e / C), c = (int)(e - (int64_t)n * C);
    float g[3][3];
#pragma unroll
    for (int t = 0; t < 9; ++t) g[t / 3][t % 3] = w[(size_t)n * ldw + t * C + c];
    wino6_filter_item(g, e, NC, U);
  }
}

// the input gradient's transform straight from the layer's ORIGINAL weights [C][9][N] (N = Cin,
// C = Cout; rotated and transposed in place, as wino4_filter_rot_tile): a block owns 32 n x 32 c
__device__ __forceinline__ void wino6_filter_rot_tile(const float* __restrict__ w, int N, int C, float* __restrict__ U,
                                                      int tile) {
  __shared__ float sg[9][32][33];  // [tap][c][n]
  const int nb = N / 32, n0 = 32 * (tile % nb), c0 = 32 * (tile / nb);
  const int tid = threadIdx.x, lx = tid & 31, ly = tid >> 5;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = ly + 8 * i;
      sg[t][c][lx] = w[((size_t)(c0 + c) * 9 + t) * N + n0 + lx];
    }
  __syncthreads();
  const int64_t NC = (int64_t)N * C;
#pragma unroll 1
  for (int i = 0; i < 4; ++i) {
    const int c = lx, nl = ly + 8 * i, n = n0 + nl;
    float g[3][3];
#pragma unroll
    for (int t = 0; t < 9; ++t) g[t / 3][t % 3] = sg[8 - t][c][nl];
    wino6_filter_item(g, (int64_t)n * C + c0 + c, NC, U);
  }
}

__global__ __launch_bounds__(256) void wino6_filter_kernel(const float* __restrict__ w, int ldw, int N, int C,
                                                           float* __restrict__ U) {
  wino6_filter_range(w, ldw, N, C, U, blockIdx.x, gridDim.x);
}
__global__ __launch_bounds__(256) void wino6_filter_rot_kernel(const float* __restrict__ w, int N, int C,
                                                               float* __restrict__ U) {
  wino6_filter_rot_tile(w, N, C, U, blockIdx.x);
}

// V[xi][t][c] = (BT d BT^T)[xi], d = the 8 x 8 input patch at rows 6 ty - 1 .., cols 6 tx - 1 ..
// (zeros past the image: padding 1 and the ragged last tiles); VW consecutive channels per thread
template <int VW>
__global__ __launch_bounds__(256) void wino6_input_kernel(const float* __restrict__ x, int ldx, int B, int H, int W,
                                                          int C, float* __restrict__ V) {
  const int c4n = C / VW, TW = (W + 5) / 6, TH = (H + 5) / 6;
  const int64_t T = (int64_t)B * TH * TW, TC = T * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < T * c4n; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t t;
    int c, b, rem;
    tile_decode<VW>(e, c4n, TH * TW, t, c, b, rem);
    const int ty = rem / TW, tx = rem - ty * TW;
    fvec<VW> v[8][8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = (fvec<VW>)0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // input row k: its row transform, then its share of every V row
      const int h = 6 * ty - 1 + k;
      fvec<VW> d[8];
#pragma unroll
      for (int l = 0; l < 8; ++l) {
        const int ww = 6 * tx - 1 + l;
        d[l] = (fvec<VW>)0.f;
        if (h >= 0 && h < H && ww >= 0 && ww < W)
          d[l] = *reinterpret_cast<const fvec<VW>*>(x + (((size_t)b * H + h) * W + ww) * ldx + c);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        fvec<VW> r = (fvec<VW>)0.f;
#pragma unroll
        for (int l = 0; l < 8; ++l) axpy_c(r, w6_bt(j, l), d[l]);
#pragma unroll
        for (int i = 0; i < 8; ++i) axpy_c(v[i][j], w6_bt(i, k), r);
      }
    }
    float* o = V + t * C + c;  // one pointer walked plane to plane
#pragma unroll
    for (int xi = 0; xi < 64; ++xi) {
      *reinterpret_cast<fvec<VW>*>(o) = v[xi / 8][xi % 8];
      o += TC;
    }
  }
}

// The same input transform at two channels per thread with HALF the accumulators (pis_tune(47, 3)):
// V rows 0..3, then 4..7, each from all eight input rows (the second pass re-reads the patch from
// L1 / L2): 8-B accesses at about half the registers of the one-pass form (212 -> ~100)
__constant__ float c_w6_bt[8][8] = {{-1.f, 0.f, 21.f / 4, 0.f, -21.f / 4, 0.f, 1.f, 0.f},
                                    {0.f, 1.f, 1.f, -17.f / 4, -17.f / 4, 1.f, 1.f, 0.f},
                                    {0.f, -1.f, 1.f, 17.f / 4, -17.f / 4, -1.f, 1.f, 0.f},
                                    {0.f, 1.f / 2, 1.f / 4, -5.f / 2, -5.f / 4, 2.f, 1.f, 0.f},
                                    {0.f, -1.f / 2, 1.f / 4, 5.f / 2, -5.f / 4, -2.f, 1.f, 0.f},
                                    {0.f, 2.f, 4.f, -5.f / 2, -5.f, 1.f / 2, 1.f, 0.f},
                                    {0.f, -2.f, 4.f, 5.f / 2, -5.f, -1.f / 2, 1.f, 0.f},
                                    {0.f, -1.f, 0.f, 21.f / 4, 0.f, -21.f / 4, 0.f, 1.f}};

__global__ __launch_bounds__(256, 4) void wino6_input2h_kernel(const float* __restrict__ x, int ldx, int B, int H, int W,
                                                            int C, float* __restrict__ V) {
  constexpr int VW = 2;
  const int c4n = C / VW, TW = (W + 5) / 6, TH = (H + 5) / 6;
  const int64_t T = (int64_t)B * TH * TW, TC = T * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < T * c4n; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t t;
    int c, b, rem;
    tile_decode<VW>(e, c4n, TH * TW, t, c, b, rem);
    const int ty = rem / TW, tx = rem - ty * TW;
#pragma unroll 1
    for (int hf = 0; hf < 2; ++hf) {  // V rows 4 hf .. 4 hf + 3 (the row factor from constant memory)
      fvec<VW> v[4][8];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = (fvec<VW>)0.f;
#pragma unroll 1
      for (int k = 0; k < 8; ++k) {
        const int h = 6 * ty - 1 + k;
        fvec<VW> d[8];
#pragma unroll
        for (int l = 0; l < 8; ++l) {
          const int ww = 6 * tx - 1 + l;
          d[l] = (fvec<VW>)0.f;
          if (h >= 0 && h < H && ww >= 0 && ww < W)
            d[l] = *reinterpret_cast<const fvec<VW>*>(x + (((size_t)b * H + h) * W + ww) * ldx + c);
        }
        float f[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) f[i] = c_w6_bt[4 * hf + i][k];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          fvec<VW> r = (fvec<VW>)0.f;
#pragma unroll
          for (int l = 0; l < 8; ++l) axpy_c(r, w6_bt(j, l), d[l]);
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i][j] += f[i] * r;
        }
      }
      float* o = V + (size_t)(32 * hf) * TC + t * C + c;
#pragma unroll
      for (int xi = 0; xi < 32; ++xi) {
        *reinterpret_cast<fvec<VW>*>(o) = v[xi / 8][xi % 8];
        o += TC;
      }
    }
  }
}

__constant__ float c_w6_at[6][8] = {{1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 1.f, 0.f},
                                    {0.f, 1.f, -1.f, 2.f, -2.f, 1.f / 2, -1.f / 2, 0.f},
                                    {0.f, 1.f, 1.f, 4.f, 4.f, 1.f / 4, 1.f / 4, 0.f},
                                    {0.f, 1.f, -1.f, 8.f, -8.f, 1.f / 8, -1.f / 8, 0.f},
                                    {0.f, 1.f, 1.f, 16.f, 16.f, 1.f / 16, 1.f / 16, 0.f},
                                    {0.f, 1.f, -1.f, 32.f, -32.f, 1.f / 32, -1.f / 32, 1.f}};

// Y = AT M AT^T per tile and VW output channels, then the direct kernels' conv epilogue on the
// outputs inside the image; POOL (g.pool): the tile's 3 x 3 max-pool outputs (6 is even: a pool
// window never straddles two tiles)
// RT (pis_tune(47, 3)): the eight M rows walked in a runtime loop (the column factor AT[i][k] from
// constant memory): the loads of one row in flight at a time, ~half the registers of the unrolled form
template <int VW, bool RT = false>
__global__ __launch_bounds__(256) void wino6_output_kernel(const float* __restrict__ Mt, IGemmArgs g, int B) {
  const int N = g.N, n4n = N / VW, TW = (g.W + 5) / 6, TH = (g.H + 5) / 6;
  const int64_t T = (int64_t)B * TH * TW, TN = T * N;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < T * n4n; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t t;
    int n, b, rem;
    tile_decode<VW>(e, n4n, TH * TW, t, n, b, rem);
    const int ty = rem / TW, tx = rem - ty * TW;
    fvec<VW> y[6][6];
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) y[i][j] = (fvec<VW>)0.f;
    const float* mp = Mt + t * N + n;  // one pointer walked plane to plane
    if constexpr (RT) {
#pragma unroll 1
      for (int k = 0; k < 8; ++k) {
        fvec<VW> m[8];
#pragma unroll
        for (int l = 0; l < 8; ++l) m[l] = *reinterpret_cast<const fvec<VW>*>(mp + (size_t)l * TN);
        mp += 8 * TN;
#pragma unroll
        for (int j = 0; j < 6; ++j) {
          fvec<VW> r = (fvec<VW>)0.f;
#pragma unroll
          for (int l = 0; l < 8; ++l) axpy_c(r, w6_at(j, l), m[l]);
#pragma unroll
          for (int i = 0; i < 6; ++i) y[i][j] += c_w6_at[i][k] * r;
        }
      }
    } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      fvec<VW> m[8];
#pragma unroll
      for (int l = 0; l < 8; ++l) {
        m[l] = *reinterpret_cast<const fvec<VW>*>(mp);
        mp += TN;
      }
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        fvec<VW> r = (fvec<VW>)0.f;
#pragma unroll
        for (int l = 0; l < 8; ++l) axpy_c(r, w6_at(j, l), m[l]);
#pragma unroll
        for (int i = 0; i < 6; ++i) axpy_c(y[i][j], w6_at(i, k), r);
      }
    }
    }
    fvec<VW> bias4 = (fvec<VW>)0.f, sc4 = (fvec<VW>)1.f;
    if (g.bias) bias4 = *reinterpret_cast<const fvec<VW>*>(g.bias + n);
    if (g.flags & PIS_SCALE) sc4 = *reinterpret_cast<const fvec<VW>*>(g.scale + (size_t)b * N + n);
    const int oy0 = 6 * ty, ox0 = 6 * tx;
#pragma unroll
    for (int qi = 0; qi < 3; ++qi) {  // row pairs 2 qi, 2 qi + 1: their epilogue, then their pooled outputs
      fvec<VW> o[2][6];
#pragma unroll
      for (int di = 0; di < 2; ++di)
#pragma unroll
        for (int j = 0; j < 6; ++j) {
          const int oy = oy0 + 2 * qi + di, ox = ox0 + j;
          o[di][j] = (fvec<VW>)0.f;
          if (oy < g.H && ox < g.W) {
            const size_t pix = ((size_t)b * g.H + oy) * g.W + ox;
            o[di][j] = conv_epilogue4<VW>(g, pix, n, y[2 * qi + di][j] + bias4, sc4);
          }
        }
      if (g.pool && oy0 + 2 * qi + 1 < g.H) {
#pragma unroll
        for (int qj = 0; qj < 3; ++qj) {
          if (ox0 + 2 * qj + 1 >= g.W) continue;
          const size_t pp = ((size_t)b * (g.H / 2) + 3 * ty + qi) * (g.W / 2) + 3 * tx + qj;
          *reinterpret_cast<fvec<VW>*>(g.pool + pp * N + n) = max4<VW>(o[0][2 * qj], o[0][2 * qj + 1], o[1][2 * qj],
                                                                      o[1][2 * qj + 1]);
        }
      }
    }
  }
}

// Many layers' filter transforms in ONE launch (pis_conv3x3_filters): one layer's grid is a few
// to a few hundred blocks, so each separate launch is latency-bound (13-47 us at C2); here every
// job's blocks run side by side. Block b belongs to the job whose [start, start + blocks) holds it.
struct FilterJobDev {
  const float* w;
  void* out;
  int N, C, dgrad, planes, blocks;
  int tile;  // 4, or 6: the F(6x6,3x3) transform U[64][N][C] (planes 0)
};
constexpr int FILTER_MAX_JOBS = 40;
struct FilterBatch {
  FilterJobDev j[FILTER_MAX_JOBS];
  int start[FILTER_MAX_JOBS + 1];
  int n;
};

__global__ __launch_bounds__(256) void wino4_filter_batch_kernel(FilterBatch fb) {
  int k = 0;
  while (k + 1 < fb.n && (int)blockIdx.x >= fb.start[k + 1]) ++k;
  const FilterJobDev& jb = fb.j[k];
  const int lb = (int)blockIdx.x - fb.start[k];
  float* U = jb.planes ? nullptr : reinterpret_cast<float*>(jb.out);
  __bf16* Up = jb.planes ? reinterpret_cast<__bf16*>(jb.out) : nullptr;
  if (jb.tile == 6) {
    if (jb.dgrad) wino6_filter_rot_tile(jb.w, jb.N, jb.C, U, lb);
    else wino6_filter_range(jb.w, 9 * jb.C, jb.N, jb.C, U, lb, jb.blocks);
  } else if (jb.planes == 2) wino4_filter_h2_wave(jb.w, 9 * jb.C, jb.N, jb.C, jb.dgrad, Up, 4 * lb + (threadIdx.x >> 6));
  else if (jb.dgrad) wino4_filter_rot_tile(jb.w, jb.N, jb.C, U, 0, Up, lb);
  else wino4_filter_range(jb.w, 9 * jb.C, jb.N, jb.C, U, 0, Up, lb, jb.blocks);
}

// V[xi][t][c] = (BT d BT^T)[xi], d = the 6x6 input patch at rows 4ty-1.., cols 4tx-1.. (zero padded)
// TM: also returns the max |V| over this item's 36 x VW values (the fused kernel's fp16x3 tile scale)
template <int VW = 4, bool TM = false>
__device__ __forceinline__ float wino4_input_item(const float* __restrict__ x, int ldx, int H, int W, int C,
                                                  float* __restrict__ V, int64_t TC, int64_t t, int b, int ty,
                                                  int tx, int c) {
  fvec<VW> v[6][6];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) v[i][j] = (fvec<VW>)0.f;
#pragma unroll
  for (int k = 0; k < 6; ++k) {  // input row k: its row transform, then its share of every V row
    const int h = 4 * ty - 1 + k;
    fvec<VW> d[6];
#pragma unroll
    for (int l = 0; l < 6; ++l) {
      const int ww = 4 * tx - 1 + l;
      d[l] = (fvec<VW>)0.f;
      if (h >= 0 && h < H && ww >= 0 && ww < W)
        d[l] = *reinterpret_cast<const fvec<VW>*>(x + (((size_t)b * H + h) * W + ww) * ldx + c);
    }
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      fvec<VW> r = (fvec<VW>)0.f;
#pragma unroll
      for (int l = 0; l < 6; ++l) axpy_c(r, w4_bt(j, l), d[l]);
#pragma unroll
      for (int i = 0; i < 6; ++i) axpy_c(v[i][j], w4_bt(i, k), r);
    }
  }
#pragma unroll
  for (int xi = 0; xi < 36; ++xi)
    *reinterpret_cast<fvec<VW>*>(V + (size_t)xi * TC + t * C + c) = v[xi / 6][xi % 6];
  float m = 0.f;
  if constexpr (TM)
#pragma unroll
    for (int xi = 0; xi < 36; ++xi)
#pragma unroll
      for (int q = 0; q < VW; ++q) m = fmaxf(m, fabsf(v[xi / 6][xi % 6][q]));
  return m;
}

// tmax[t][c / 64] = max |V| over the tile's 64-channel chunk: 64 / VW consecutive lanes (C % 64 ==
// 0, so a chunk's lanes are an aligned group of one wave and take the same grid-stride trip count).
// The fp16x3 consumers take one power-of-two scale per tile (row) from the max over its chunks.
template <int VW>
__device__ __forceinline__ void tile_max_store(float m, int C, int c, int64_t t, float* __restrict__ tmax) {
#pragma unroll
  for (int off = 32 / VW; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
  if ((c & 63) == 0) tmax[t * (C >> 6) + (c >> 6)] = m;
}

// VW channels per thread (pis_tune key 17): 2 (default) = half the registers of 4 (float4 accesses)
template <int VW, bool TM = false>
__global__ __launch_bounds__(256) void wino4_input_kernel(const float* __restrict__ x, int ldx, int B, int H, int W,
                                                          int C, float* __restrict__ V,
                                                          float* __restrict__ tmax = nullptr) {
  const int c4n = C / VW, TW = W / 4, TH = H / 4;
  const int64_t T = (int64_t)B * TH * TW, TC = T * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < T * c4n; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t t;
    int c, b, rem;
    tile_decode<VW>(e, c4n, TH * TW, t, c, b, rem);
    const int ty = rem / TW, tx = rem - ty * TW;
    const float m = wino4_input_item<VW, TM>(x, ldx, H, W, C, V, TC, t, b, ty, tx, c);
    if constexpr (TM) tile_max_store<VW>(m, C, c, t, tmax);
  }
}

// Y = AT M AT^T per tile and VW output channels (pis_tune key 17), then the direct kernels' conv
// epilogue. MPF (input gradients with a ReLU mask, pis_tune key 46): the tile's 16 mask rows are
// loaded with its M values, so the epilogue does not wait for a second memory round trip.
template <int VW, bool MPF = false>
__global__ __launch_bounds__(256) void wino4_output_kernel(const float* __restrict__ Mt, IGemmArgs g, int B) {
  const int N = g.N, n4n = N / VW, TW = g.W / 4, TH = g.H / 4;
  const int64_t T = (int64_t)B * TH * TW, TN = T * N;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < T * n4n; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t t;
    int n, b, rem;
    tile_decode<VW>(e, n4n, TH * TW, t, n, b, rem);
    const int ty = rem / TW, tx = rem - ty * TW;
    fvec<VW> mk[4][4];
    if constexpr (MPF) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const size_t pix = ((size_t)b * g.H + 4 * ty + i) * g.W + 4 * tx + j;
          mk[i][j] = *reinterpret_cast<const fvec<VW>*>(g.mask + pix * g.ldm + n);
        }
    }
    fvec<VW> y[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) y[i][j] = (fvec<VW>)0.f;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      fvec<VW> m[6];
#pragma unroll
      for (int l = 0; l < 6; ++l) m[l] = *reinterpret_cast<const fvec<VW>*>(Mt + (size_t)(k * 6 + l) * TN + t * N + n);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        fvec<VW> r = (fvec<VW>)0.f;
#pragma unroll
        for (int l = 0; l < 6; ++l) axpy_c(r, w4_at(j, l), m[l]);
#pragma unroll
        for (int i = 0; i < 4; ++i) axpy_c(y[i][j], w4_at(i, k), r);
      }
    }
    fvec<VW> bias4 = (fvec<VW>)0.f, sc4 = (fvec<VW>)1.f;
    if (g.bias) bias4 = *reinterpret_cast<const fvec<VW>*>(g.bias + n);
    if (g.flags & PIS_SCALE) sc4 = *reinterpret_cast<const fvec<VW>*>(g.scale + (size_t)b * N + n);
    fvec<VW> o[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const size_t pix = ((size_t)b * g.H + 4 * ty + i) * g.W + 4 * tx + j;
        if constexpr (MPF) o[i][j] = conv_epilogue_vm<VW>(g, pix, n, y[i][j] + bias4, sc4, mk[i][j]);
        else o[i][j] = conv_epilogue4<VW>(g, pix, n, y[i][j] + bias4, sc4);
      }
    if (g.pool) {  // the tile's four 2x2 max-pool outputs (the encoder's MaxPool2d)
#pragma unroll
      for (int qi = 0; qi < 2; ++qi)
#pragma unroll
        for (int qj = 0; qj < 2; ++qj) {
          const size_t pp = ((size_t)b * (g.H / 2) + 2 * ty + qi) * (g.W / 2) + 2 * tx + qj;
          *reinterpret_cast<fvec<VW>*>(g.pool + pp * N + n) =
              max4<VW>(o[2 * qi][2 * qj], o[2 * qi][2 * qj + 1], o[2 * qi + 1][2 * qj], o[2 * qi + 1][2 * qj + 1]);
        }
    }
  }
}

// ---- weight gradient F(3x3, 4x4): 4x4 output-gradient tiles, 36 contractions over tiles ----
// dW[r] = sum_k x[4t - 1 + r + k] dz[4t + k] per tile is the correlation F(3, 4): 6 input
// samples, 4 "filter" taps (the dz tile), 3 outputs (the weight taps). Same points
// {0, 1, -1, 1/2, -2, inf}, so the input transform is the forward's BT (wino4_input_kernel);
// E = G4 e G4^T with G4 (6x4), dW = AT3 M AT3^T with AT3 (3x6). fp32 error 1.3e-6 relative
// (F(3x3,2x2): 0.4e-6, direct 0.6e-6; 256-channel layers against float64).
__host__ __device__ constexpr float w4_g4(int i, int k) {
  constexpr float m[6][4] = {{1.f, 0.f, 0.f, 0.f},
                             {1.f / 3, 1.f / 3, 1.f / 3, 1.f / 3},
                             {-1.f / 3, 1.f / 3, -1.f / 3, 1.f / 3},
                             {-16.f / 15, -8.f / 15, -4.f / 15, -2.f / 15},
                             {1.f / 15, -2.f / 15, 4.f / 15, -8.f / 15},
                             {0.f, 0.f, 0.f, 1.f}};
  return m[i][k];
}
__host__ __device__ constexpr float w4_at3(int i, int k) {
  constexpr float m[3][6] = {{1.f, 1.f, 1.f, 1.f, 1.f, 0.f},
                             {0.f, 1.f, -1.f, 0.5f, -2.f, 0.f},
                             {0.f, 1.f, 1.f, 0.25f, 4.f, 1.f}};
  return m[i][k];
}

// E[xi][t][n] = (G4 e G4^T)[xi], e = dz at output pixels (4ty + i, 4tx + j); bsum += the tile's
// channel sums (the bias gradient)
template <int VW = 4>
__device__ __forceinline__ void wino4_dz_item(const float* __restrict__ dz, int ldz, int H, int W, int N,
                                              float* __restrict__ E, int64_t TN, int64_t t, int b, int ty, int tx,
                                              int n, fvec<VW>& bsum) {
  fvec<VW> v[6][6];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) v[i][j] = (fvec<VW>)0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    fvec<VW> d[4];
#pragma unroll
    for (int l = 0; l < 4; ++l)
      d[l] = *reinterpret_cast<const fvec<VW>*>(dz + (((size_t)b * H + 4 * ty + k) * W + 4 * tx + l) * ldz + n);
    bsum += (d[0] + d[1]) + (d[2] + d[3]);
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      fvec<VW> r = (fvec<VW>)0.f;
#pragma unroll
      for (int l = 0; l < 4; ++l) axpy_c(r, w4_g4(j, l), d[l]);
#pragma unroll
      for (int i = 0; i < 6; ++i) axpy_c(v[i][j], w4_g4(i, k), r);
    }
  }
#pragma unroll
  for (int xi = 0; xi < 36; ++xi)
    *reinterpret_cast<fvec<VW>*>(E + (size_t)xi * TN + t * N + n) = v[xi / 6][xi % 6];
}

// bpart[blockIdx.x][N] = fixed-order block reduction of the threads sharing a channel group
// (tid mod N / VW; with 256 a multiple of N / VW a thread's channels never change across its
// grid-stride items)
template <int VW = 4>
__device__ __forceinline__ void wino4_bias_partials(fvec<VW> bsum, int N, float* __restrict__ bpart) {
  const int nvn = N / VW;
  __shared__ fvec<VW> red[256];
  red[threadIdx.x] = bsum;
  __syncthreads();
  if ((int)threadIdx.x < nvn) {
    fvec<VW> acc = red[threadIdx.x];
    for (int k = threadIdx.x + nvn; k < 256; k += nvn) acc += red[k];
    *reinterpret_cast<fvec<VW>*>(bpart + (size_t)blockIdx.x * N + VW * threadIdx.x) = acc;
  }
}

// With bpart != NULL it also leaves the bias gradient's per-block channel sums in
// bpart[blockIdx.x][N] (every dz pixel belongs to exactly one tile).
template <int VW = 4>
__global__ __launch_bounds__(256) void wino4_dz_kernel(const float* __restrict__ dz, int ldz, int B, int H, int W,
                                                       int N, float* __restrict__ E, float* __restrict__ bpart) {
  const int nvn = N / VW, TW = W / 4, TH = H / 4;
  const int64_t T = (int64_t)B * TH * TW, TN = T * N;
  fvec<VW> bsum = (fvec<VW>)0.f;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < T * nvn; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t t;
    int n, b, rem;
    tile_decode<VW>(e, nvn, TH * TW, t, n, b, rem);
    const int ty = rem / TW, tx = rem - ty * TW;
    wino4_dz_item<VW>(dz, ldz, H, W, N, E, TN, t, b, ty, tx, n, bsum);
  }
  if (bpart) wino4_bias_partials<VW>(bsum, N, bpart);
}

// One pass over a layer's dz for both of its backward products: V = the input gradient's
// F(4x4,3x3) input transform of dz (as wino4_input_kernel) and E = the weight gradient's
// F(3x3,4x4) transform + bias partials (as wino4_dz_kernel); the second half re-reads the tile's
// 4x4 interior from cache instead of HBM. Same grid as wino4_dz_kernel (bpart layout).
// VW channels per thread (dz_vw: 2 where 256 is a multiple of N / 2, so the bias partials keep
// one channel pair per thread; half the registers of the float4 form, whose 256 + 30 kept it at one
// wave per SIMD)
template <bool TM = false, int VW = 4>
__global__ __launch_bounds__(256) void wino4_dz2_kernel(const float* __restrict__ dz, int ldz, int B, int H, int W,
                                                        int N, float* __restrict__ V, float* __restrict__ E,
                                                        float* __restrict__ bpart, float* __restrict__ tmax = nullptr) {
  const int nvn = N / VW, TW = W / 4, TH = H / 4;
  const int64_t T = (int64_t)B * TH * TW, TN = T * N;
  fvec<VW> bsum = (fvec<VW>)0.f;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < T * nvn; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t t;
    int n, b, rem;
    tile_decode<VW>(e, nvn, TH * TW, t, n, b, rem);
    const int ty = rem / TW, tx = rem - ty * TW;
    const float m = wino4_input_item<VW, TM>(dz, ldz, H, W, N, V, TN, t, b, ty, tx, n);
    if constexpr (TM) tile_max_store<VW>(m, N, n, t, tmax);
    wino4_dz_item<VW>(dz, ldz, H, W, N, E, TN, t, b, ty, tx, n, bsum);
  }
  if (bpart) wino4_bias_partials<VW>(bsum, N, bpart);
}

// dw[n][r][s][c] (+)= (AT3 M AT3^T)[r][s], M[xi][n][c] the reduced tile sums
// M may arrive as `nsplit` split-K slabs `sstride` floats apart (summed here in slab order,
// which saves the separate slab reduction's write + re-read of the 36 planes)
__global__ __launch_bounds__(256) void wino4_wgrad_out_kernel(const float* __restrict__ M, int N, int C,
                                                              float* __restrict__ dw, int accumulate, int nsplit,
                                                              int64_t sstride) {
  const int64_t NC = (int64_t)N * C;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < NC; e += (int64_t)gridDim.x * blockDim.x) {
    const int n = (int)(e / C), c = (int)(e - (int64_t)n * C);
    float y[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) y[i][j] = 0.f;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      float m[6];
#pragma unroll
      for (int l = 0; l < 6; ++l) {
        const float* src = M + (size_t)(k * 6 + l) * NC + e;
        float v = src[0];
        for (int sp = 1; sp < nsplit; ++sp) v += src[sp * sstride];
        m[l] = v;
      }
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        float r = 0.f;
#pragma unroll
        for (int l = 0; l < 6; ++l) axpy_c(r, w4_at3(j, l), m[l]);
#pragma unroll
        for (int i = 0; i < 3; ++i) axpy_c(y[i][j], w4_at3(i, k), r);
      }
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        float* o = dw + ((size_t)n * 9 + i * 3 + j) * C + c;
        *o = accumulate ? *o + y[i][j] : y[i][j];
      }
  }
}

// the folded bias gradient (WgradOutBias) of the output transforms' first nb blocks: 256 channels
// per block, every thread one channel summed over the partial rows in a fixed order
__device__ __forceinline__ void wgrad_out_bias_block(int N, int accumulate, const WgradOutBias& bias) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const float* pp = bias.part + n;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;  // four chains, combined in a fixed order
  int r = 0;
  for (; r + 3 < bias.rows; r += 4) {
    s0 += pp[(size_t)r * N];
    s1 += pp[(size_t)(r + 1) * N];
    s2 += pp[(size_t)(r + 2) * N];
    s3 += pp[(size_t)(r + 3) * N];
  }
  for (; r < bias.rows; ++r) s0 += pp[(size_t)r * N];
  const float v = ((s0 + s1) + (s2 + s3)) * bias.scale;
  bias.db[n] = accumulate ? bias.db[n] + v : v;
}

// The same as a block-tiled pass (NC % 64 == 0: every F(3x3,4x4) layer with 64-multiple channels).
// The one-thread-per-(n, c) form above ran at 0.7 TB/s in the step (profiles/r4_e: 36 x nsplit
// dependent-latency loads per thread, 256 blocks of 256 threads for a 256 x 256 layer). Here a
// block owns 64 consecutive (n, c): pass 1 sums the split slabs of its 36 x 64 M entries, 9 per
// thread, 4 slabs per unrolled step so 36 loads are in flight, into LDS; pass 2 runs the output
// transform with 3 threads per entry (one row i of the 3 x 3 each). Same sums in the same order as
// wino4_wgrad_out_kernel: bitwise equal.
// The first nb blocks are the bias gradient's (WgradOutBias): 256 channels each, every thread one
// channel summed over the partial rows in order, so the weight gradient's bias costs no launch.
__global__ __launch_bounds__(256) void wino4_wgrad_out_tiled_kernel(const float* __restrict__ M, int N, int C,
                                                                    float* __restrict__ dw, int accumulate,
                                                                    int nsplit, int64_t sstride, WgradOutBias bias,
                                                                    int nb) {
  if ((int)blockIdx.x < nb) {
    wgrad_out_bias_block(N, accumulate, bias);
    return;
  }
  __shared__ float sm[36][65];
  const int64_t NC = (int64_t)N * C;
  const int64_t e0 = (int64_t)(blockIdx.x - nb) * 64;
  const int tid = threadIdx.x, el = tid & 63, xg = tid >> 6;  // entry e0 + el, xi = xg + 4 q
  {
    const float* src[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) src[q] = M + (size_t)(xg + 4 * q) * NC + e0 + el;
    float v[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) v[q] = src[q][0];
    int sp = 1;
    for (; sp + 3 < nsplit; sp += 4) {
      float a[9][4];
#pragma unroll
      for (int q = 0; q < 9; ++q)
#pragma unroll
        for (int u = 0; u < 4; ++u) a[q][u] = src[q][(size_t)(sp + u) * sstride];
#pragma unroll
      for (int q = 0; q < 9; ++q) v[q] = (((v[q] + a[q][0]) + a[q][1]) + a[q][2]) + a[q][3];
    }
    for (; sp < nsplit; ++sp)
#pragma unroll
      for (int q = 0; q < 9; ++q) v[q] += src[q][(size_t)sp * sstride];
#pragma unroll
    for (int q = 0; q < 9; ++q) sm[xg + 4 * q][el] = v[q];
  }
  __syncthreads();
  if (tid >= 192) return;
  const int i = tid >> 6;  // output row r = i of entry el
  float y[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    float m[6];
#pragma unroll
    for (int l = 0; l < 6; ++l) m[l] = sm[k * 6 + l][el];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float r = 0.f;
#pragma unroll
      for (int l = 0; l < 6; ++l) axpy_c(r, w4_at3(j, l), m[l]);
      const float a = i == 0 ? w4_at3(0, k) : i == 1 ? w4_at3(1, k) : w4_at3(2, k);
      if (a == 1.f) y[j] += r;
      else if (a == -1.f) y[j] -= r;
      else if (a != 0.f) y[j] += a * r;  // as axpy_c (contracted to the same fma)
    }
  }
  const int64_t e = e0 + el;
  const int n = (int)(e / C), c = (int)(e - (int64_t)n * C);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    float* o = dw + ((size_t)n * 9 + i * 3 + j) * C + c;
    *o = accumulate ? *o + y[j] : y[j];
  }
}

// wino4_wgrad_out_tiled_kernel with 16-B lanes (pis_tune key 48 = 1, default; C % 4 == 0). The
// scalar form moved 256 B per wave load over 36 x nsplit strided rows and ran at 1.14 TB/s
// (71.6 MB in 62.7 us per launch, profiles/r5_final2). Here a block owns EPB = 64 / 128 / 256
// consecutive (n, c) entries; pass 1: each lane sums the split slabs of 4 consecutive entries of
// plane rows xi = xg, xg + G, ... (EPB / 4 lanes per row, G = 1024 / EPB rows at a time, two
// slabs per unrolled step: up to 18 float4 loads in flight, 1 KB per wave load at EPB = 256);
// pass 2: 3 EPB / 4 lanes, each one output row i of 4 entries, float4 LDS reads and dw stores.
// Same sums in the same order per element: bitwise equal to the scalar forms.
template <int EPB>
__global__ __launch_bounds__(256) void wino4_wgrad_out_v4_kernel(const float* __restrict__ M, int N, int C,
                                                                 float* __restrict__ dw, int accumulate, int nsplit,
                                                                 int64_t sstride, WgradOutBias bias, int nb) {
  constexpr int L = EPB / 4, G = 256 / L, Q = (36 + G - 1) / G;
  if ((int)blockIdx.x < nb) {  // the bias gradient, as wino4_wgrad_out_tiled_kernel
    wgrad_out_bias_block(N, accumulate, bias);
    return;
  }
  __shared__ __attribute__((aligned(16))) float sm[36][EPB + 4];
  const int64_t NC = (int64_t)N * C;
  const int64_t e0 = (int64_t)(blockIdx.x - nb) * EPB;
  const int tid = threadIdx.x, l4 = tid % L, xg = tid / L;
  {
    const float* src[Q];
    f32x4 v[Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const int xi = xg + G * q;
      src[q] = M + (size_t)(xi < 36 ? xi : 0) * NC + e0 + 4 * l4;
      v[q] = xi < 36 ? *reinterpret_cast<const f32x4*>(src[q]) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    int sp = 1;
    for (; sp + 1 < nsplit; sp += 2) {
      f32x4 a[Q][2];
#pragma unroll
      for (int q = 0; q < Q; ++q)
#pragma unroll
        for (int u = 0; u < 2; ++u)
          if (xg + G * q < 36) a[q][u] = *reinterpret_cast<const f32x4*>(src[q] + (size_t)(sp + u) * sstride);
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (xg + G * q < 36) v[q] = (v[q] + a[q][0]) + a[q][1];
    }
    for (; sp < nsplit; ++sp)
#pragma unroll
      for (int q = 0; q < Q; ++q)
        if (xg + G * q < 36) v[q] += *reinterpret_cast<const f32x4*>(src[q] + (size_t)sp * sstride);
#pragma unroll
    for (int q = 0; q < Q; ++q)
      if (xg + G * q < 36) *reinterpret_cast<f32x4*>(&sm[xg + G * q][4 * l4]) = v[q];
  }
  __syncthreads();
  if (tid >= 3 * L) return;
  const int i = tid / L, e4 = tid % L;  // output row r = i of entries 4 e4 .. 4 e4 + 3
  f32x4 y[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) y[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    f32x4 m[6];
#pragma unroll
    for (int l = 0; l < 6; ++l) m[l] = *reinterpret_cast<const f32x4*>(&sm[k * 6 + l][4 * e4]);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      f32x4 r = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int l = 0; l < 6; ++l) axpy_c(r, w4_at3(j, l), m[l]);
      const float a = i == 0 ? w4_at3(0, k) : i == 1 ? w4_at3(1, k) : w4_at3(2, k);
      if (a == 1.f) y[j] += r;
      else if (a == -1.f) y[j] -= r;
      else if (a != 0.f) y[j] += a * r;
    }
  }
  const int64_t e = e0 + 4 * e4;
  const int n = (int)(e / C), c = (int)(e - (int64_t)n * C);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    f32x4* o = reinterpret_cast<f32x4*>(dw + ((size_t)n * 9 + i * 3 + j) * C + c);
    *o = accumulate ? *o + y[j] : y[j];
  }
}

// ---- the batched GEMMs (16 or 36): C[z][m][n] = sum_k A[z][m][k] B[z][n][k] ------------
// Both operands K-contiguous ("NT"), plain row-major C, no epilogue: a lean kernel for the
// Winograd contractions. Block tile BM x BN (4 waves, 2 x 2, each (BM/2) x (BN/2) as 32x32 MFMA
// tiles), K-step 16 through a register-staged LDS double buffer; LDS rows padded to 20 floats
// so the 16-byte fragment reads are conflict-free; one ds_read_b128 feeds 4 MFMAs.
// (BK = 32 measured within +-3 % of BK = 16 on every Winograd layer: tools/bench_kernels.py --key 10)
template <int BM, int BN, int BK = 16>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(const float* __restrict__ A, const float* __restrict__ Bm,
                                                        float* __restrict__ Cm, int M, int N, int K,
                                                        int64_t bsA, int64_t bsB, int64_t bsC) {
  constexpr int ROW = BK + 4, CPR = BK / 4;  // LDS row pitch; float4 chunks per staged row
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int AL = BM * CPR / 256, BL = BN * CPR / 256;  // float4 loads per thread per stage
  __shared__ __attribute__((aligned(16))) float sA[2][BM * ROW];
  __shared__ __attribute__((aligned(16))) float sB[2][BN * ROW];
  const Remap2 rm = xcd_remap2();
  A += rm.batch * bsA;
  Bm += rm.batch * bsB;
  Cm += rm.batch * bsC;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, lh = lane >> 5;
  const int ntn = N / BN;
  const int bid = rm.bid;
  const int m0 = (bid / ntn) * BM, n0 = (bid % ntn) * BN;
  const int q4 = (tid % CPR) * 4;
  f32x4 ra[AL], rb[BL];
  auto gload = [&](int k0) {
    const int k = k0 + q4;
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int m = m0 + (tid + i * 256) / CPR;
      ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (m < M && k < K) ra[i] = *reinterpret_cast<const f32x4*>(A + (size_t)m * K + k);
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int n = n0 + (tid + i * 256) / CPR;
      rb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (k < K) rb[i] = *reinterpret_cast<const f32x4*>(Bm + (size_t)n * K + k);
    }
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < AL; ++i) *reinterpret_cast<f32x4*>(&sA[buf][((tid + i * 256) / CPR) * ROW + q4]) = ra[i];
#pragma unroll
    for (int i = 0; i < BL; ++i) *reinterpret_cast<f32x4*>(&sB[buf][((tid + i * 256) / CPR) * ROW + q4]) = rb[i];
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const int KT = (K + BK - 1) / BK;
  gload(0);
  lstore(0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) gload((kt + 1) * BK);
#pragma unroll
    for (int gg = 0; gg < BK / 8; ++gg) {
      f32x4 af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a)
        af[a] = *reinterpret_cast<const f32x4*>(&sA[cur][(wm * (BM / 2) + a * 32 + li) * ROW + 8 * gg + 4 * lh]);
#pragma unroll
      for (int b = 0; b < TN; ++b)
        bf[b] = *reinterpret_cast<const f32x4*>(&sB[cur][(wn * (BN / 2) + b * 32 + li) * ROW + 8 * gg + 4 * lh]);
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
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int n = n0 + wn * (BN / 2) + b * 32 + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * (BM / 2) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) Cm[(size_t)m * N + n] = acc[a][b][r];
      }
    }
}

// ---- the same GEMMs at fp32 accuracy on bf16 MFMA ("bf16x6") ----------------------------
// Each fp32 operand is split exactly into hi + mid + lo bf16 (hi = bf16(x), mid = bf16(x - hi),
// lo = bf16(x - hi - mid): 24 significant bits); a product needs the six partial products with
// order <= 2^-24 of the largest (hi.hi, hi.mid, mid.hi, hi.lo, mid.mid, lo.hi), which bf16 MFMA
// forms exactly and accumulates in fp32. v_mfma_f32_32x32x16_bf16 retires 16x the FLOPs of
// v_mfma_f32_32x32x2_f32 per cycle, so the six cost 6/16 of one fp32 MFMA pass. Measured error
// (CPU emulation, 128-1024-deep products): 0.9-1.4e-7 relative, below native fp32's 2-3.4e-7.
// The split happens once per staged element (global -> LDS), not per MFMA use.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));


// DBG (timing only, wrong results): 1 no global loads, 2 no split.
template <int BM, int BN, int DBG = 0>
__global__ __launch_bounds__(256, 2) void gemm_nt_x6_kernel(
    const float* __restrict__ A, const float* __restrict__ Bm, float* __restrict__ Cm, int M, int N, int K,
    int64_t bsA, int64_t bsB, int64_t bsC) {
  constexpr int BK = 16;
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int AL = BM * 4 / 256, BL = BN * 4 / 256;  // float4 loads per thread per stage
  __shared__ __attribute__((aligned(16))) __bf16 sA[2][3][BM * BK];  // [buf][hi|mid|lo][row][k]
  __shared__ __attribute__((aligned(16))) __bf16 sB[2][3][BN * BK];
  const Remap2 rm = xcd_remap2();
  A += rm.batch * bsA;
  Bm += rm.batch * bsB;
  Cm += rm.batch * bsC;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, lh = lane >> 5;
  const int ntn = N / BN;
  const int bid = rm.bid;
  const int m0 = (bid / ntn) * BM, n0 = (bid % ntn) * BN;
  const int q4 = (tid & 3) * 4;
  const bool full = m0 + BM <= M && K % BK == 0;
  struct Regs {
    f32x4 a[AL], b[BL];
  };
  auto gload = [&](int k0, Regs& r) {
    const int k = k0 + q4;
    if (DBG == 1) {
#pragma unroll
      for (int i = 0; i < AL; ++i) r.a[i] = f32x4{(float)k0, 1.f, 2.f, 3.f};
#pragma unroll
      for (int i = 0; i < BL; ++i) r.b[i] = f32x4{(float)k0, 1.f, 2.f, 3.f};
      return;
    }
    if (full) {  // block-uniform: no per-load guards (exec masking) inside the tile
#pragma unroll
      for (int i = 0; i < AL; ++i)
        r.a[i] = *reinterpret_cast<const f32x4*>(A + (size_t)(m0 + (tid + i * 256) / 4) * K + k);
    } else {
#pragma unroll
      for (int i = 0; i < AL; ++i) {
        const int m = m0 + (tid + i * 256) / 4;
        r.a[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (m < M && k < K) r.a[i] = *reinterpret_cast<const f32x4*>(A + (size_t)m * K + k);
      }
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int n = n0 + (tid + i * 256) / 4;
      r.b[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (full || k < K) r.b[i] = *reinterpret_cast<const f32x4*>(Bm + (size_t)n * K + k);
    }
  };
  auto split = [&](f32x4 v, u32x2& h, u32x2& m, u32x2& l) {
    if (DBG == 2) {
      h = u32x2{__builtin_bit_cast(unsigned, v[0]), __builtin_bit_cast(unsigned, v[2])};
      m = h;
      l = h;
    } else {
      split3_x4(v, h, m, l);
    }
  };
  auto lstore = [&](int buf, const Regs& r) {
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      u32x2 h, m, l;
      split(r.a[i], h, m, l);
      const int o = ((tid + i * 256) / 4) * BK + q4;
      *reinterpret_cast<u32x2*>(&sA[buf][0][o]) = h;
      *reinterpret_cast<u32x2*>(&sA[buf][1][o]) = m;
      *reinterpret_cast<u32x2*>(&sA[buf][2][o]) = l;
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      u32x2 h, m, l;
      split(r.b[i], h, m, l);
      const int o = ((tid + i * 256) / 4) * BK + q4;
      *reinterpret_cast<u32x2*>(&sB[buf][0][o]) = h;
      *reinterpret_cast<u32x2*>(&sB[buf][1][o]) = m;
      *reinterpret_cast<u32x2*>(&sB[buf][2][o]) = l;
    }
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  auto compute = [&](int cur) {
    bf16x8 af[3][TM], bf[3][TN];  // lane: row li, k = 8 lh .. 8 lh + 7
#pragma unroll
    for (int p = 0; p < 3; ++p) {
#pragma unroll
      for (int a = 0; a < TM; ++a)
        af[p][a] = *reinterpret_cast<const bf16x8*>(&sA[cur][p][(wm * (BM / 2) + a * 32 + li) * BK + 8 * lh]);
#pragma unroll
      for (int b = 0; b < TN; ++b)
        bf[p][b] = *reinterpret_cast<const bf16x8*>(&sB[cur][p][(wn * (BN / 2) + b * 32 + li) * BK + 8 * lh]);
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
  };
  const int KT = (K + BK - 1) / BK;
  Regs x;
  gload(0, x);
  lstore(0, x);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) gload((kt + 1) * BK, x);
    compute(cur);
    if (kt + 1 < KT) lstore(cur ^ 1, x);
    __syncthreads();
  }
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int n = n0 + wn * (BN / 2) + b * 32 + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * (BM / 2) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) Cm[(size_t)m * N + n] = acc[a][b][r];
      }
    }
}

// K-step 32 variant of gemm_nt_x6_kernel with ONE LDS buffer (48 KB at 128 x 128, so three
// blocks still fit a CU): compute, barrier, store the next stage, barrier, issue the loads of
// the stage after — a load has a whole 48-MFMA compute phase to land, and every 128-B line a
// wave touches is consumed in the same stage. LDS rows are 64 B (32 bf16) with the 16-B chunk
// XOR-swizzled by row bits 2..3 (x6w8_off): conflict-free ds_read_b128 fragments AND ds_write_b64
// staging (two rows = 128 contiguous bytes), and 48 KB per 128 x 128 block, so three blocks fit a
// CU (80-B padded rows: 60 KB, two blocks, and 2-way conflicted staging stores).
template <int BM, int BN, int OCC = 2>
__global__ __launch_bounds__(256, OCC) void gemm_nt_x6_bk32_kernel(const float* __restrict__ A,
                                                                const float* __restrict__ Bm, float* __restrict__ Cm,
                                                                int M, int N, int K, int64_t bsA, int64_t bsB,
                                                                int64_t bsC) {
  constexpr int BK = 32, KP = 32;
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int AL = BM * 8 / 256, BL = BN * 8 / 256;  // float4 loads per thread per stage
  __shared__ __attribute__((aligned(16))) __bf16 sA[3][BM * KP];
  __shared__ __attribute__((aligned(16))) __bf16 sB[3][BN * KP];
  const Remap2 rm = xcd_remap2();
  A += rm.batch * bsA;
  Bm += rm.batch * bsB;
  Cm += rm.batch * bsC;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, lh = lane >> 5;
  const int ntn = N / BN;
  const int bid = rm.bid;
  const int m0 = (bid / ntn) * BM, n0 = (bid % ntn) * BN;
  const int q8 = (tid & 7) * 4;
  const bool full = m0 + BM <= M && K % BK == 0;
  f32x4 ra[AL], rb[BL];
  auto gload = [&](int k0) {
    const int k = k0 + q8;
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int m = m0 + (tid + i * 256) / 8;
      ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (full || (m < M && k < K)) ra[i] = *reinterpret_cast<const f32x4*>(A + (size_t)m * K + k);
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int n = n0 + (tid + i * 256) / 8;
      rb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (full || k < K) rb[i] = *reinterpret_cast<const f32x4*>(Bm + (size_t)n * K + k);
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      u32x2 h, m, l;
      split3_x4(ra[i], h, m, l);
      const int row = (tid + i * 256) / 8, o = x6w8_off(row, q8 >> 3) + (q8 & 7);
      *reinterpret_cast<u32x2*>(&sA[0][o]) = h;
      *reinterpret_cast<u32x2*>(&sA[1][o]) = m;
      *reinterpret_cast<u32x2*>(&sA[2][o]) = l;
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      u32x2 h, m, l;
      split3_x4(rb[i], h, m, l);
      const int row = (tid + i * 256) / 8, o = x6w8_off(row, q8 >> 3) + (q8 & 7);
      *reinterpret_cast<u32x2*>(&sB[0][o]) = h;
      *reinterpret_cast<u32x2*>(&sB[1][o]) = m;
      *reinterpret_cast<u32x2*>(&sB[2][o]) = l;
    }
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const int KT = (K + BK - 1) / BK;
  gload(0);
  lstore();
  if (KT > 1) gload(BK);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 af[3][TM], bf[3][TN];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
#pragma unroll
        for (int a = 0; a < TM; ++a)
          af[p][a] = *reinterpret_cast<const bf16x8*>(&sA[p][x6w8_off(wm * (BM / 2) + a * 32 + li, 2 * ks + lh)]);
#pragma unroll
        for (int b = 0; b < TN; ++b)
          bf[p][b] = *reinterpret_cast<const bf16x8*>(&sB[p][x6w8_off(wn * (BN / 2) + b * 32 + li, 2 * ks + lh)]);
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
    }
    if (kt + 1 < KT) {
      __syncthreads();
      lstore();
      __syncthreads();
      if (kt + 2 < KT) gload((kt + 2) * BK);
    }
  }
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int n = n0 + wn * (BN / 2) + b * 32 + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * (BM / 2) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (m < M) Cm[(size_t)m * N + n] = acc[a][b][r];
      }
    }
}

// ---- fp16x3: hi/lo fp16 split, 3 products, in the bk32 structure ---------------
// 2 planes per operand (2/3 of bf16x6's LDS) and half its MFMAs; each K-step's tiles scaled by
// a power of two into fp16 range (SC; the unscaled form is pis_debug_gemm_nt variant 10 only).
// Scales per WAVE and K-step: the 8 threads that stage one 32-k row of a tile belong to one wave
// (row = tid / 8 + 32 i), so each wave scales the rows it stages by the power of two of its own
// maximum (no block-wide exchange: no extra barrier), and publishes it in LDS with the planes.
// In the 32 x 32 MFMA output a lane holds column n = li (B row staged by wave (li / 8) % 4) and
// rows r -> (r & 3) + 8 (r >> 2) + 4 lh (A rows staged by wave r >> 2): accumulator register r
// is in units sA[r >> 2] * sB[(li / 8) % 4], and is re-expressed when a K-step's scales differ.
//
// (An epilogue through LDS — 16-B row pieces, 4 rows x 256 B per wave store — measured neutral to
// -2 % per layer, profiles/r3_q18_gemm_le.txt; the wave index is made scalar: no VGPR spill.)
// DBG (timing twins, pis_debug_gemm_nt variants 13 / 14, wrong results): 1 no global loads after the
// first two K-steps, 2 no staging after the first (profiles/r3_q22_gemm_twins.txt: staging is 24-44 %
// of the time, the loads 0-17 %). (Two LDS stages + two register sets at two blocks per CU — one
// barrier per K-step, loads a K-step further ahead — ran 10-30 % slower: profiles/r3_q23_gemm_db.txt.)
template <int BM, int BN, int OCC = 3, bool SC = true, int DBG = 0>
__global__ __launch_bounds__(256, OCC) void gemm_nt_h3_bk32_kernel(const float* __restrict__ A,
                                                                const float* __restrict__ Bm, float* __restrict__ Cm,
                                                                int M, int N, int K, int64_t bsA, int64_t bsB,
                                                                int64_t bsC) {
  constexpr int BK = 32, KP = 32;
  constexpr bool WS = SC;  // per-wave, per-K-step scales
  constexpr int TM = BM / 64, TN = BN / 64;
  constexpr int AL = BM * 8 / 256, BL = BN * 8 / 256;
  static_assert(BM % 128 == 0 && BN % 64 == 0, "row r's staging wave must be r / 8 % 4");
  __shared__ __attribute__((aligned(16))) _Float16 smem[2 * (BM + BN) * KP];
  _Float16(*sA)[BM * KP] = reinterpret_cast<_Float16(*)[BM * KP]>(smem);
  _Float16(*sB)[BN * KP] = reinterpret_cast<_Float16(*)[BN * KP]>(smem + 2 * BM * KP);
  __shared__ __attribute__((aligned(16))) float sscale[2][4];  // [A|B][staging wave]
  const Remap2 rm = xcd_remap2();
  A += rm.batch * bsA;
  Bm += rm.batch * bsB;
  Cm += rm.batch * bsC;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1, li = lane & 31, lh = lane >> 5;
  const int ntn = N / BN;
  const int bid = rm.bid;
  const int m0 = (bid / ntn) * BM, n0 = (bid % ntn) * BN;
  const int q8 = (tid & 7) * 4;
  const bool full = m0 + BM <= M && K % BK == 0;
  f32x4 ra[AL], rb[BL];
  // full tiles (every launch of the training step): straight-line buffer loads from the block's
  // first A / B row (SGPR resources), one 32-bit lane offset for both operands (row tid / 8,
  // column q8) and a wave-uniform offset per row group i and K-step; rows of one block tile span
  // BM * K * 4 bytes (< 2 GiB for any K the host admits)
  const __amdgpu_buffer_rsrc_t rsa =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A + (size_t)m0 * K), (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(Bm + (size_t)n0 * K), (short)0, 0x7fffffff, 0x00020000);
  const uint32_t vo = 4u * ((uint32_t)(tid / 8) * (uint32_t)K + (uint32_t)q8);
  auto gload = [&](int k0) {
    if (DBG == 1 && k0 >= 2 * BK) return;
    if (full) {
#pragma unroll
      for (int i = 0; i < AL; ++i)
        ra[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsa, vo, 4u * (uint32_t)(32 * i * K + k0), 0));
#pragma unroll
      for (int i = 0; i < BL; ++i)
        rb[i] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsb, vo, 4u * (uint32_t)(32 * i * K + k0), 0));
      return;
    }
    const int k = k0 + q8;
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int m = m0 + (tid + i * 256) / 8;
      ra[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (m < M && k < K) ra[i] = *reinterpret_cast<const f32x4*>(A + (size_t)m * K + k);
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int n = n0 + (tid + i * 256) / 8;
      rb[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (k < K) rb[i] = *reinterpret_cast<const f32x4*>(Bm + (size_t)n * K + k);
    }
  };
  float sa = 0.f, sb = 0.f;  // the wave's current scales (h3_keep)
  float sa_min = __builtin_inff(), sb_min = __builtin_inff();  // ... and the smallest so far
  auto lstore = [&]() {
    if (WS) {
      sa = h3_keep(sa, wave_max_nonneg(absmax_x4(ra)), sa_min);
      sb = h3_keep(sb, wave_max_nonneg(absmax_x4(rb)), sb_min);
      if (lane == 0) {
        sscale[0][wave] = sa;
        sscale[1][wave] = sb;
      }
    }
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      u32x2 h, l;
      split2h_x4(WS ? ra[i] * sa : ra[i], h, l);
      const int row = (tid + i * 256) / 8, o = x6w8_off(row, q8 >> 3) + (q8 & 7);
      *reinterpret_cast<u32x2*>(&sA[0][o]) = h;
      *reinterpret_cast<u32x2*>(&sA[1][o]) = l;
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      u32x2 h, l;
      split2h_x4(WS ? rb[i] * sb : rb[i], h, l);
      const int row = (tid + i * 256) / 8, o = x6w8_off(row, q8 >> 3) + (q8 & 7);
      *reinterpret_cast<u32x2*>(&sB[0][o]) = h;
      *reinterpret_cast<u32x2*>(&sB[1][o]) = l;
    }
  };
  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const int KT = (K + BK - 1) / BK;
  gload(0);
  lstore();
  if (KT > 1) gload(BK);
  __syncthreads();
  f32x4 ua = {1.f, 1.f, 1.f, 1.f};  // units of the accumulators: A scale per row group r >> 2,
  float ub = 1.f;                   // B scale of this lane's column
  for (int kt = 0; kt < KT; ++kt) {
    if (WS) {  // this K-step's scales; re-express the partial sums in them (exact: powers of two)
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
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[a][b][r] *= f[r >> 2];
        ua = na;
        ub = nb;
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      f16x8 af[2][TM], bf[2][TN];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
#pragma unroll
        for (int a = 0; a < TM; ++a)
          af[p][a] = *reinterpret_cast<const f16x8*>(&sA[p][x6w8_off(wm * (BM / 2) + a * 32 + li, 2 * ks + lh)]);
#pragma unroll
        for (int b = 0; b < TN; ++b)
          bf[p][b] = *reinterpret_cast<const f16x8*>(&sB[p][x6w8_off(wn * (BN / 2) + b * 32 + li, 2 * ks + lh)]);
      }
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[1][a], bf[0][b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0][a], bf[1][b], acc[a][b], 0, 0, 0);
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[0][a], bf[0][b], acc[a][b], 0, 0, 0);
        }
    }
    if (kt + 1 < KT) {
      __syncthreads();
      if (DBG != 2) lstore();
      __syncthreads();
      if (kt + 2 < KT) gload((kt + 2) * BK);
    }
  }
  float inv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) inv[q] = WS ? 1.f / (ua[q] * ub) : 1.f;
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int nl = wn * (BN / 2) + b * 32 + li, n = n0 + nl;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ml = wm * (BM / 2) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh, m = m0 + ml;
        if (m < M) Cm[(size_t)m * N + n] = acc[a][b][r] * inv[r >> 2];
      }
    }
}

// ---- F(4x4,3x3) contraction fused with the output transform (bf16x6) --------------------
// For the shallow, HBM-bound layers: the 36 products M[xi] = V[xi] U[xi]^T never go to HBM.
// A block owns TB = 16 NWT tiles x all N = 16 NWN output channels (V is read exactly once) and
// walks xi = 0..35; wave (wt, wn) computes the 16 x 16 product of tiles 16 wt.. and channels
// 16 wn.. on v_mfma_f32_16x16x32_bf16 (bf16x6, fp32 accumulation) and folds it straight into
// Y = AT M AT^T: per row a of the 6x6 grid the lane keeps R[j] = sum_b AT[j][b] M[a][b], then
// Y[i][j] += AT[i][a] R[j] — 16 x 4 accumulators per lane (lane l: channel l & 15 of tiles
// 4 (l >> 4) .. + 3). Per xi both operands are staged in LDS: V[xi] (TB x KC fp32, one
// contiguous run) is loaded RING stages ahead into registers and split into hi/mid/lo at the
// LDS store; U[xi] arrives pre-split (wino4_filter_kernel Up planes, L2-resident) and is copied
// with coalesced 16-B loads two stages ahead. One barrier per xi. Then the direct kernels'
// epilogue (bias, ReLU, mask, keep-scale, accumulate).
typedef __bf16 bf16x8g __attribute__((ext_vector_type(8)));

// H3: fp16x3 instead (pis_tune key 22). Every V row (tile) is split into hi / lo fp16 of v * s_t
// with ONE power of two s_t per tile for all 36 xi and 64 channels, from the tile's max |V| that
// the V producer wrote (wino4_input_kernel / wino4_dz2_kernel `tmax`), and the filter planes carry
// one scale t_n per output channel (wino4_filter_h2_*): M[xi] and therefore Y are in units
// s_t t_n for every xi, so the products need no per-xi unscaling — the epilogue divides once.
// Elements more than 2^16 below their tile's max keep an absolute error <= 2^-37 of that max,
// far below the fp32 transform's own rounding (~2^-24 of the patch max). One chain of three fp16
// products (lo hi, hi lo, hi hi) per K-step: two thirds of the LDS operand reads, half the MFMAs.
// STG (pis_tune key 25): the second half of the waves (wt = 1: the SIMD partners of waves 0-3)
// fold each xi's product one xi late, keeping it in registers across the barrier (a stagger,
// MI355X_MICROARCH.md 'Two waves that run the SAME program with one barrier per block'): the
// partners' MFMA and fold phases no longer coincide. Bit-for-bit the same sums in the same order.
template <int NWN, int NWT, int KC, int G = 1, bool H3 = false, bool STG = false>
__global__ __launch_bounds__(64 * NWN * NWT) void wino4_gemm_out_x6_kernel(const float* __restrict__ V,
                                                                          const __bf16* __restrict__ Up,
                                                                          IGemmArgs g, int B,
                                                                          const float* __restrict__ tmax = nullptr) {
  constexpr int NT = 64 * NWN * NWT, TB = 16 * NWT, NN = 16 * NWN, KP = KC;  // KP: LDS row pitch (bf16)
  constexpr int P = H3 ? 2 : 3;  // operand planes
  // unpadded rows, 16-B chunks XOR-swizzled by (row / 2) % 8: every ds_read_b128 lane group (16
  // rows of one 16-row window, two adjacent chunks) hits 16 distinct slots of the 256-B bank row;
  // without the 8-element padding a block needs 72 KB of LDS, so two blocks share a CU
  // KC = 128 (128-channel contractions): 256-B rows span a whole bank row, so the 16-B chunk is
  // XOR-swizzled by the row's low 4 bits (16 rows of one ds_read_b128 lane group: 16 slots)
  static_assert(KC == 64 || KC == 128, "the swizzle spans 8 or 16 chunks of 8 bf16");
  auto sw = [](int row, int k) {
    const int x = KC == 64 ? (row >> 1) & 7 : row & 15;
    return row * KP + ((((k >> 3) ^ x) << 3) | (k & 7));
  };
  constexpr int NV4 = TB * KC / 4, AL = (NV4 + NT - 1) / NT;  // float4 of V[xi] per thread
  constexpr bool VPART = NV4 % NT != 0;                         // (then NV4 < NT: some threads idle)
  constexpr int NU8 = P * NN * KC / 8, UL = NU8 / NT;          // 16-B chunks of the U[xi] planes per thread
  static_assert((!VPART || NV4 < NT) && NU8 % NT == 0, "staging must tile the block");
  // V stages in flight: 6 x 8 KB (KC = 64) or 3 x 16 KB (KC = 128); 10 stages in the staggered
  // KC = 64 form (it has the registers) measured 2 % slower (profiles/r2_q82_*)
  constexpr int RING = KC == 64 ? 6 : 3, KS = KC / 32;
  // LDS: the double-buffered operand planes, and (aliased) the epilogue's staging of all four
  // tile quarters of Y (139 KB: one block per CU either way, its registers allow no second)
  constexpr int QT = 4 * NWT, EP = NN + 4, EQ = QT * 16 * EP;  // tiles per quarter; row pitch, floats
  constexpr int NB = 2;  // LDS operand buffers
  constexpr int OPS_BYTES = NB * P * (TB + NN) * KP * 2, EPI_BYTES = 4 * EQ * 4;
  constexpr int LDS_BYTES = OPS_BYTES > EPI_BYTES ? OPS_BYTES : EPI_BYTES;
  static_assert(QT * 4 * (NN / 4) == NT, "one epilogue item per thread and quarter");
  static_assert(!H3 || (AL <= 2 && !VPART), "H3: at most two V rows per thread (their tile scales in registers)");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  auto sA = reinterpret_cast<__bf16(*)[P][TB * KP]>(smem);
  auto sU = reinterpret_cast<__bf16(*)[P][NN * KP]>(smem + NB * P * TB * KP * 2);
  float* E = reinterpret_cast<float*>(smem);
  const int N = g.N, TW = g.W / 4, TH = g.H / 4;
  const int64_t T = (int64_t)B * TH * TW;
  int64_t TK = T * KC, NK = (int64_t)N * KC;  // laundered per group with Ug (below)
  int tid = threadIdx.x;  // laundered per group (below), like every tid-derived address
  const int lane = tid & 63, wave = tid >> 6;
  const int wn = wave % NWN, wt = wave / NWN;
  const int lr = lane & 15, lq = lane >> 4;
  const int n = 16 * wn + lr;  // this lane's output channel within the block's NN
  // N > NN (pis_tune key 26): nblk blocks share a tile group, one NN-channel slice each, dealt
  // so that they sit 8 apart in dispatch order (one XCD, back to back: V comes from its L2)
  const int nblk = N / NN;
  int gblk = blockIdx.x, nb = 0;
  if (nblk > 1) {
    if ((gridDim.x / nblk) % 8 == 0) {
      gblk = (blockIdx.x / (8 * nblk)) * 8 + blockIdx.x % 8;
      nb = (blockIdx.x / 8) % nblk;
    } else {
      gblk = blockIdx.x / nblk;
      nb = blockIdx.x % nblk;
    }
  }
  const int n0 = nb * NN;
  // G consecutive groups of TB tiles per block: the next group's first V and U loads are issued
  // before this group's epilogue, so their latency hides behind its stores
  const int64_t grp0 = (int64_t)gblk * G;
  f32x4 vr[RING][AL];
  auto gload = [&](const float* vb, int xi, f32x4 (&r)[AL]) {
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      // wave-uniform base + unsigned 32-bit per-thread byte offset (a buffer load): no per-load
      // 64-bit VALU address arithmetic
      if (!VPART || tid + i * NT < NV4)
        r[i] = __builtin_bit_cast(f32x4, buf_load16(vb + xi * TK, 16u * (uint32_t)(tid + i * NT)));
    }
  };
  auto lstore = [&](int buf, const f32x4 (&r)[AL], f32x2 srow) {  // srow: H3 tile scales of the rows
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int idx = tid + i * NT;
      if (VPART && idx >= NV4) continue;
      const int row = idx / (KC / 4), c = 4 * (idx % (KC / 4));
      if constexpr (H3) {
        u32x2 h, l;
        split2h_x4(r[i] * srow[i], h, l);
        *reinterpret_cast<u32x2*>(&sA[buf][0][sw(row, c)]) = h;
        *reinterpret_cast<u32x2*>(&sA[buf][1][sw(row, c)]) = l;
        continue;
      }
      u32x2 h, m, l;
      split3_x4(r[i], h, m, l);
      *reinterpret_cast<u32x2*>(&sA[buf][0][sw(row, c)]) = h;
      *reinterpret_cast<u32x2*>(&sA[buf][1][sw(row, c)]) = m;
      *reinterpret_cast<u32x2*>(&sA[buf][P - 1][sw(row, c)]) = l;
    }
  };
  u32x4 ur[2][UL];
  const __bf16* Ug = Up;  // laundered per group (below): keeps 36 x UL U addresses from being hoisted
  auto uload = [&](int xi, int slot) {
#pragma unroll
    for (int i = 0; i < UL; ++i) {
      const int c = tid + i * NT;  // (plane, channel, 8-k chunk), k fastest: contiguous per plane
      const int pl = c / (NN * KC / 8), rem = c % (NN * KC / 8);
      // (a buffer load from a uniform base, like gload: global, not FLAT, so it stays out of lgkmcnt
      // and LDS waits do not wait for its L2 round trip)
      ur[slot][i] = buf_load16(Ug + xi * NK + n0 * KC, 2u * ((uint32_t)pl * 36u * (uint32_t)NK + 8u * (uint32_t)rem));
    }
  };
  auto ustore = [&](int buf, int slot) {
#pragma unroll
    for (int i = 0; i < UL; ++i) {
      const int c = tid + i * NT;
      const int pl = c / (NN * KC / 8), rem = c % (NN * KC / 8);
      const int row = rem / (KC / 8), k = 8 * (rem % (KC / 8));
      *reinterpret_cast<u32x4*>(&sU[buf][pl][sw(row, k)]) = ur[slot][i];
    }
  };
  // a group's first stages: V[0..RING) and U[0..2) in flight, V[0] / U[0] in LDS buffer 0
  auto prime = [&](const float* vb) {
#pragma unroll
    for (int j = 0; j < RING; ++j) gload(vb, j, vr[j]);
  };
  auto first_stage = [&](const float* vb, f32x2 srow) {
    uload(0, 0);
    uload(1, 1);
    lstore(0, vr[0], srow);
    ustore(0, 0);
    gload(vb, RING, vr[0]);
    uload(2, 0);
    __syncthreads();
  };
  // H3: this thread's V row is tile t0 + tid / (KC / 4) of each group (AL == 1); its scale, and the
  // inverse scale of this lane's output channel n (after the two filter planes)
  auto tile_scale = [&](float m) {
    float sc, inv;
    h2_scale_pair(m, sc, inv);
    return sc;
  };
  // a tile's max |V| over its KC / 64 channel chunks (tmax[t][KC / 64])
  auto tmx = [&](int64_t t) {
    float m = tmax[t * (KC / 64)];
#pragma unroll
    for (int j = 1; j < KC / 64; ++j) m = fmaxf(m, tmax[t * (KC / 64) + j]);
    return m;
  };
  // the tile maxima of this thread's staged rows (row = (tid + i NT) / (KC / 4)) in group t0
  auto row_max = [&](int64_t t0) {
    f32x2 m = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < AL; ++i) m[i] = tmx(t0 + (tid + i * NT) / (KC / 4));
    return m;
  };
  auto row_scale = [&](f32x2 m) { return f32x2{tile_scale(m[0]), tile_scale(m[1])}; };
  f32x2 srow = {1.f, 1.f}, tm_next = {0.f, 0.f};
  if constexpr (H3) srow = row_scale(row_max(grp0 * TB));
  prime(V + grp0 * TB * KC);
  first_stage(V + grp0 * TB * KC, srow);
#pragma unroll 1
  for (int gi = 0; gi < G; ++gi) {
    const int64_t t0 = (grp0 + gi) * TB;
    const float* vb = V + t0 * KC;
    // two statements: an asm whose outputs include a VGPR is divergent as a whole, and the buffer
    // loads need Ug / TK / NK wave-uniform
    asm volatile("" : "+s"(Ug), "+s"(TK), "+s"(NK));
    asm volatile("" : "+v"(tid));
    f32x4 y[4][4], rr[4], accp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      rr[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 4; ++j) y[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const bool late = STG && wt == 1;  // wave-uniform
    // Y[i][j] += AT[i][ra] R[j], then R = 0 (ra: the grid row whose six products R holds)
    auto rowend = [&](int ra) {
      float at[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = 0.f;
#pragma unroll
        for (int q = 0; q < 6; ++q) v = ra == q ? w4_at(i, q) : v;
        at[i] = v;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) y[i][j] += at[i] * rr[j];
#pragma unroll
      for (int j = 0; j < 4; ++j) rr[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    };
#pragma unroll
    for (int a = 0; a < 6; ++a) {  // fully unrolled: the compiler keeps exact vmcnt counts across rows
#pragma unroll
      for (int b = 0; b < 6; ++b) {
        const int xi = 6 * a + b, cur = b & 1;
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        if constexpr (H3) {
#pragma unroll
          for (int s = 0; s < KS; ++s) {
            const int k = 32 * s + 8 * lq;
            const f16x8 a0 = *reinterpret_cast<const f16x8*>(&sA[cur][0][sw(16 * wt + lr, k)]);
            const f16x8 a1 = *reinterpret_cast<const f16x8*>(&sA[cur][1][sw(16 * wt + lr, k)]);
            const f16x8 b0 = *reinterpret_cast<const f16x8*>(&sU[cur][0][sw(n, k)]);
            const f16x8 b1 = *reinterpret_cast<const f16x8*>(&sU[cur][1][sw(n, k)]);
            // smallest partial products first
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b0, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b1, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b0, acc, 0, 0, 0);
          }
        }
#pragma unroll
        for (int s = 0; s < (H3 ? 0 : KS); ++s) {
          const int k = 32 * s + 8 * lq;
          bf16x8g af[3], bf[3];
#pragma unroll
          for (int p = 0; p < 3; ++p) {
            af[p] = *reinterpret_cast<const bf16x8g*>(&sA[cur][p % P][sw(16 * wt + lr, k)]);
            bf[p] = *reinterpret_cast<const bf16x8g*>(&sU[cur][p % P][sw(n, k)]);
          }
          // smallest partial products first
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[2], bf[0], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], bf[1], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bf[2], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1], bf[0], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bf[1], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0], bf[0], acc, 0, 0, 0);
        }
        if (!late) {
#pragma unroll
          for (int j = 0; j < 4; ++j) axpy_c(rr[j], w4_at(j, b), acc);
        } else {  // fold the previous xi's product (column b - 1, or the previous row's last)
          if (xi > 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) axpy_c(rr[j], w4_at(j, (b + 5) % 6), accp);
            if (b == 0) rowend(a - 1);
          }
          accp = acc;
        }
        // stage xi + 1 (V from its ring slot, U from the register pair), then refill both
        const int vslot = (xi + 1) % RING;
        if (xi + 1 < 36) {
          lstore(cur ^ 1, vr[vslot], srow);
          ustore(cur ^ 1, cur ^ 1);
        }
        if (xi + 1 + RING < 36) gload(vb, xi + 1 + RING, vr[vslot]);
        if (xi + 3 < 36) uload(xi + 3, cur ^ 1);
        __syncthreads();
      }
      // Y[i][j] += AT[i][a] R[j] (a is a runtime row index: coefficients selected from the table)
      if (!late) rowend(a);
    }
    if (late) {  // the last product
#pragma unroll
      for (int j = 0; j < 4; ++j) axpy_c(rr[j], w4_at(j, 5), accp);
      rowend(5);
    }
    const bool more = gi + 1 < G;
    if (more) {
      if constexpr (H3) tm_next = row_max(t0 + TB);
      prime(vb + TB * KC);
    }
    if constexpr (H3) {
      // Y is in units s_t t_n: divide (exact powers of two, one factor at a time)
      const float inv_t = reinterpret_cast<const float*>(Up + 2 * 36 * (int64_t)N * KC)[n0 + n];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float sc, inv_s;
        h2_scale_pair(tmx(t0 + 16 * wt + 4 * lq + q), sc, inv_s);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) y[i][j][q] = (y[i][j][q] * inv_s) * inv_t;
      }
    }
    // epilogue: the lanes' (channel n, tiles t0 + 16 wt + 4 lq + q) values of all four tile
    // quarters q go through LDS so that every thread finishes 4 consecutive channels of one 2x2
    // pixel quad per quarter with float4 accesses; its ReLU-mask loads for the four quads are
    // issued together, before the barrier (one memory round trip per group, not four)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) E[q * EQ + ((4 * wt + lq) * 16 + 4 * i + j) * EP + n] = y[i][j][q];
    int et = tid;  // laundered: the epilogue's index math stays out of the group loop's registers
    asm volatile("" : "+v"(et));
    const int c4 = et % (NN / 4), pq = et / (NN / 4);
    const int tl = pq / 4, quad = pq % 4, qi = quad >> 1, qj = quad & 1, nl = 4 * c4, nn = n0 + nl;
    size_t pix0[4], pp[4];  // the quad's first pixel; its pooled pixel
    int bq[4];
    f32x4 mk[4][2][2];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t t = t0 + 16 * (tl / 4) + 4 * (tl % 4) + q;
      const int b = (int)(t / (TH * TW)), rem = (int)(t - (int64_t)b * TH * TW);
      const int ty = rem / TW, tx = rem - ty * TW;
      bq[q] = b;
      pix0[q] = ((size_t)b * g.H + 4 * ty + 2 * qi) * g.W + 4 * tx + 2 * qj;
      pp[q] = ((size_t)b * (g.H / 2) + 2 * ty + qi) * (g.W / 2) + 2 * tx + qj;
#pragma unroll
      for (int di = 0; di < 2; ++di)
#pragma unroll
        for (int dj = 0; dj < 2; ++dj)
          mk[q][di][dj] = (g.flags & PIS_MASK)
                              ? *reinterpret_cast<const f32x4*>(g.mask + (pix0[q] + di * g.W + dj) * g.ldm + nn)
                              : f32x4{1.f, 1.f, 1.f, 1.f};
    }
    __syncthreads();
    f32x4 bias4 = {0.f, 0.f, 0.f, 0.f};
    if (g.bias) bias4 = *reinterpret_cast<const f32x4*>(g.bias + nn);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f32x4 sc4 = {1.f, 1.f, 1.f, 1.f};
      if (g.flags & PIS_SCALE) sc4 = *reinterpret_cast<const f32x4*>(g.scale + (size_t)bq[q] * N + nn);
      f32x4 o[2][2];
#pragma unroll
      for (int di = 0; di < 2; ++di)
#pragma unroll
        for (int dj = 0; dj < 2; ++dj) {
          const int i = 2 * qi + di, j = 2 * qj + dj;
          const f32x4 v = *reinterpret_cast<const f32x4*>(&E[q * EQ + (tl * 16 + 4 * i + j) * EP + nl]);
          o[di][dj] = conv_epilogue4m(g, pix0[q] + di * g.W + dj, nn, v + bias4, sc4, mk[q][di][dj]);
        }
      if (g.pool) *reinterpret_cast<f32x4*>(g.pool + pp[q] * N + nn) = max4(o[0][0], o[0][1], o[1][0], o[1][1]);
    }
    __syncthreads();
    if (more) {
      if constexpr (H3) srow = row_scale(tm_next);
      first_stage(vb + TB * KC, srow);
    }
  }
}

static int grid_of(int64_t work) { return (int)std::max<int64_t>(1, std::min<int64_t>(cdiv(work, 256), 16384)); }

// the F(4x4,3x3) output transform, 2 (default) or 4 channels per thread (pis_tune key 17;
// tools/bench_kernels.py --key 17: 2 channels halve the registers, +2-11 % on the 512^2-256^2 layers)
static void launch_wino4_output(const float* Mt, const IGemmArgs& a, int B, int64_t T, int N, hipStream_t s) {
  if (tune_get(PIS_TUNE_WINO_VW) != 4)
    if ((a.flags & PIS_MASK) && a.mask && tune_get(PIS_TUNE_WINO_OUT_MPF) != 0)
      hipLaunchKernelGGL((wino4_output_kernel<2, true>), dim3(grid_of(T * (N / 2))), dim3(256), 0, s, Mt, a, B);
    else
      hipLaunchKernelGGL(wino4_output_kernel<2>, dim3(grid_of(T * (N / 2))), dim3(256), 0, s, Mt, a, B);
  else
    hipLaunchKernelGGL(wino4_output_kernel<4>, dim3(grid_of(T * (N / 4))), dim3(256), 0, s, Mt, a, B);
}

// the F(4x4,3x3) input transform, 2 (default) or 4 channels per thread (pis_tune key 17)
// tmax (C % 64 == 0): also the per-tile, per-64-channel-chunk max |V| (the fp16x3 tile scales)
static void launch_wino4_input(int64_t T, int C, hipStream_t s, const float* x, int ldx, int B, int H, int W, int,
                               float* V, float* tmax = nullptr) {
  const bool vw2 = tune_get(PIS_TUNE_WINO_VW) != 4;
  if (tmax && vw2)
    hipLaunchKernelGGL((wino4_input_kernel<2, true>), dim3(grid_of(T * (C / 2))), dim3(256), 0, s, x, ldx, B, H, W, C,
                       V, tmax);
  else if (tmax)
    hipLaunchKernelGGL((wino4_input_kernel<4, true>), dim3(grid_of(T * (C / 4))), dim3(256), 0, s, x, ldx, B, H, W, C,
                       V, tmax);
  else if (vw2)
    hipLaunchKernelGGL(wino4_input_kernel<2>, dim3(grid_of(T * (C / 2))), dim3(256), 0, s, x, ldx, B, H, W, C, V,
                       nullptr);
  else
    hipLaunchKernelGGL(wino4_input_kernel<4>, dim3(grid_of(T * (C / 4))), dim3(256), 0, s, x, ldx, B, H, W, C, V,
                       nullptr);
}

// the F(4x4,3x3) filter transform of a's weights (the tiled kernel for unflipped 32-aligned shapes)
// (Up: the fused kernel's planes, bf16x6 or, with h2, fp16x3 + scales — C % 32 == 0)
static void launch_wino4_filter(const IGemmArgs& a, int N, int C, float* U, int transposed, __bf16* Up,
                                hipStream_t s, bool h2 = false) {
  if (h2)  // C % 64 == 0, N % 4 == 0 (the fused kernel's shapes)
    hipLaunchKernelGGL(wino4_filter_h2_kernel, dim3(N / 4), dim3(256), 0, s, a.wt, a.ldw, N, C, a.w_unflipped ? 1 : 0,
                       Up);
  else if (a.w_unflipped)  // N, C % 32 == 0 checked by launch_wino3x3
    hipLaunchKernelGGL(wino4_filter_rot_kernel, dim3((N / 32) * (C / 32)), dim3(256), 0, s, a.wt, N, C, U,
                       transposed, Up);
  else
    hipLaunchKernelGGL(wino4_filter_kernel, dim3(grid_of((int64_t)N * C)), dim3(256), 0, s, a.wt, a.ldw, N, C, U,
                       transposed, Up);
}

// the fused 64 -> 64 kernel's arithmetic (pis_tune key 22): fp16x3 planes instead of bf16x6
static bool wino_gemm_out_h3() { return tune_get(PIS_TUNE_WINO_GEMM_OUT_H3) != 0; }

// fused path eligibility (pis_tune key 15): F(4x4), bf16x6 GEMMs, 64 -> 64 channels. Measured
// (tools/bench_kernels.py --key 15, C2): enc1.conv1 forward 1.13 -> 0.98 ms, input gradient
// 1.30 -> 1.13 ms; with 128 input or output channels (dec1.conv0, enc2.conv0) it is 2-8 % slower
// than the separate GEMM + output transform, so those keep the 3-pass pipeline.
static bool wino_gemm_out_wanted(int m, int64_t T, int C, int N) {
  // N = 128 (64-channel contractions into 128 outputs: enc2.conv0 forward, dec1.conv0 input
  // gradient) with pis_tune key 26: two blocks per tile group, V read twice (from L2), M never
  return m == 4 && tune_get(PIS_TUNE_WINO_GEMM_OUT) != 0 && tune_get(PIS_TUNE_WINO_TILE) >= 3 && T % 32 == 0 &&
         T >= 2 * (int64_t)C &&  // the filter planes fit in the M region
         (C == 64 || (C == 128 && tune_get(PIS_TUNE_FUSED_K128) != 0)) &&
         (N == 64 || (N % 64 == 0 && N <= 64 * (1 << tune_get(PIS_TUNE_FUSED_WIDE))));
}

static int launch_wino_gemm_out(const float* V, const __bf16* Up, const IGemmArgs& a, int B, int64_t T,
                                hipStream_t s, const float* tmax) {
  // 8 waves: 32 tiles x 64 channels per block; G such groups per block where they divide
  // (pis_tune key 15: 1 -> G = 4, 2 -> 1, 3 -> 2, 4 -> 8: experiments)
  const int64_t groups = T / 32;
  const int nblk = a.N / 64;  // 64-channel slices (pis_tune key 26: N = 128 too)
  const int mode = tune_get(PIS_TUNE_WINO_GEMM_OUT);
  const int G = mode == 2 ? 1 : mode == 3 ? 2 : mode == 4 ? 8 : 4;
  const dim3 blk(512);
  if (a.Csrc == 128) {
    // KC = 128 always staggered where it can be: that form fits 250 VGPRs, the lockstep one spills
    if (wino_gemm_out_h3() && groups % 4 == 0) {
      hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 128, 4, true, true>), dim3((int)(groups / 4) * nblk), blk, 0, s, V, Up,
                         a, B, tmax);
    } else if (wino_gemm_out_h3()) {
      if (G == 8 && groups % 8 == 0)
        hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 128, 8, true>), dim3((int)(groups / 8) * nblk), blk, 0, s, V, Up, a,
                           B, tmax);
      else if (G == 4 && groups % 4 == 0)
        hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 128, 4, true>), dim3((int)(groups / 4) * nblk), blk, 0, s, V, Up, a,
                           B, tmax);
      else if (G == 2 && groups % 2 == 0)
        hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 128, 2, true>), dim3((int)(groups / 2) * nblk), blk, 0, s, V, Up, a,
                           B, tmax);
      else
        hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 128, 1, true>), dim3((int)groups * nblk), blk, 0, s, V, Up, a, B, tmax);
    } else if (G == 8 && groups % 8 == 0)
      hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 128, 8>), dim3((int)(groups / 8) * nblk), blk, 0, s, V, Up, a, B, nullptr);
    else if (G == 4 && groups % 4 == 0)
      hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 128, 4>), dim3((int)(groups / 4) * nblk), blk, 0, s, V, Up, a, B, nullptr);
    else if (G == 2 && groups % 2 == 0)
      hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 128, 2>), dim3((int)(groups / 2) * nblk), blk, 0, s, V, Up, a, B, nullptr);
    else
      hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 128, 1>), dim3((int)groups * nblk), blk, 0, s, V, Up, a, B, nullptr);
  } else {
  if (wino_gemm_out_h3() && tune_get(PIS_TUNE_FUSED_STAGGER) != 0 && groups % 4 == 0) {
      hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 64, 4, true, true>), dim3((int)(groups / 4) * nblk), blk, 0, s, V, Up,
                         a, B, tmax);
    } else if (wino_gemm_out_h3()) {
      if (G == 8 && groups % 8 == 0)
        hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 64, 8, true>), dim3((int)(groups / 8) * nblk), blk, 0, s, V, Up, a,
                           B, tmax);
      else if (G == 4 && groups % 4 == 0)
        hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 64, 4, true>), dim3((int)(groups / 4) * nblk), blk, 0, s, V, Up, a,
                           B, tmax);
      else if (G == 2 && groups % 2 == 0)
        hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 64, 2, true>), dim3((int)(groups / 2) * nblk), blk, 0, s, V, Up, a,
                           B, tmax);
      else
        hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 64, 1, true>), dim3((int)groups * nblk), blk, 0, s, V, Up, a, B, tmax);
    } else if (G == 8 && groups % 8 == 0)
      hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 64, 8>), dim3((int)(groups / 8) * nblk), blk, 0, s, V, Up, a, B, nullptr);
    else if (G == 4 && groups % 4 == 0)
      hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 64, 4>), dim3((int)(groups / 4) * nblk), blk, 0, s, V, Up, a, B, nullptr);
    else if (G == 2 && groups % 2 == 0)
      hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 64, 2>), dim3((int)(groups / 2) * nblk), blk, 0, s, V, Up, a, B, nullptr);
    else
      hipLaunchKernelGGL((wino4_gemm_out_x6_kernel<4, 2, 64, 1>), dim3((int)groups * nblk), blk, 0, s, V, Up, a, B, nullptr);
  }
  return launch_status("wino_gemm_out");
}


// does a contraction of C channels into N outputs at B x H x W take the fused F(4x4) kernel?
bool wino_fused_wanted(int B, int H, int W, int C, int N) {
  return wino_tile(H, W) == 4 && wino_gemm_out_wanted(4, (int64_t)B * (H / 4) * (W / 4), C, N);
}

static int64_t wino6_tiles(int B, int H, int W) { return (int64_t)B * ((H + 5) / 6) * ((W + 5) / 6); }

// U (64 N C), V (64 T C), M (64 T N) of one F(6x6,3x3) call
static size_t wino6_ws_bytes(int B, int H, int W, int C, int N) {
  const int64_t T = wino6_tiles(B, H, W);
  return (size_t)64 * ((int64_t)N * C + T * C + T * N) * sizeof(float) + 1024;
}

// the F(6x6,3x3) filter transform of w: forward weights [N][9][C] (ldw), or (dgrad) the input
// gradient's from the ORIGINAL weights [C][9][N] (N, C % 32 == 0)
static void launch_wino6_filter(const float* w, int ldw, int N, int C, int dgrad, float* U, hipStream_t s) {
  if (dgrad) hipLaunchKernelGGL(wino6_filter_rot_kernel, dim3((N / 32) * (C / 32)), dim3(256), 0, s, w, N, C, U);
  else hipLaunchKernelGGL(wino6_filter_kernel, dim3(grid_of((int64_t)N * C)), dim3(256), 0, s, w, ldw, N, C, U);
}

int launch_wino6_filter_only(const float* w, int C, int N, int dgrad, void* out, hipStream_t s) {
  if (dgrad && (N % 32 || C % 32))
    return set_error("pis_conv3x3_filter: the F(6x6) input-gradient transform needs 32-aligned channels"), PIS_ERR_ARG;
  launch_wino6_filter(w, 9 * C, N, C, dgrad, reinterpret_cast<float*>(out), s);
  return launch_status("wino6_filter");
}

// one F(6x6,3x3) convolution (a: as launch_wino3x3): filter transform (or a.wt ready: U[64][N][C]),
// input transform, the 64 batched fp16x3 GEMMs, output transform + epilogue
static int launch_wino6(const IGemmArgs& a, int B, void* ws, hipStream_t s) {
  const int C = a.Csrc, N = a.N;
  const int64_t T = wino6_tiles(B, a.H, a.W);
  float* U = (float*)ws;
  float* V = U + (size_t)64 * N * C;
  float* Mt = V + (size_t)64 * T * C;
  if (a.w_unflipped && (N % 32 || C % 32))
    return set_error("launch_wino6: unflipped weights need 32-aligned channels"), PIS_ERR_ARG;
  if (a.filter_ready) U = const_cast<float*>(a.wt);
  else launch_wino6_filter(a.wt, a.ldw, N, C, a.w_unflipped ? 1 : 0, U, s);
  // channels per thread of the transforms (key 47: 1 -> 1, 2 -> 2): the 64-value tiles hold 64 VW
  // accumulators per thread
  const int f6 = tune_get(PIS_TUNE_WINO_F6);
  const bool vw2 = f6 == 2;
  if (f6 == 3)
    hipLaunchKernelGGL(wino6_input2h_kernel, dim3(grid_of(T * (C / 2))), dim3(256), 0, s, a.src, a.lds, B, a.H, a.W,
                       C, V);
  else if (vw2)
    hipLaunchKernelGGL(wino6_input_kernel<2>, dim3(grid_of(T * (C / 2))), dim3(256), 0, s, a.src, a.lds, B, a.H, a.W,
                       C, V);
  else
    hipLaunchKernelGGL(wino6_input_kernel<1>, dim3(grid_of(T * C)), dim3(256), 0, s, a.src, a.lds, B, a.H, a.W, C, V);
  int rc = launch_status("wino6_transforms");
  if (rc) return rc;
  const double flop = 2.0 * 64 * (double)T * N * C;
  launch_hook("wino_gemm", 0, s, flop);
  if (N % 128 == 0) {
    const dim3 grid((int)cdiv(T, 128) * (N / 128), 64);
    hipLaunchKernelGGL((gemm_nt_h3_bk32_kernel<128, 128, 3>), grid, dim3(256), 0, s, V, U, Mt, (int)T, N, C, T * C,
                       (int64_t)N * C, T * N);
  } else {
    const dim3 grid((int)cdiv(T, 128) * (N / 64), 64);
    hipLaunchKernelGGL((gemm_nt_h3_bk32_kernel<128, 64, 4>), grid, dim3(256), 0, s, V, U, Mt, (int)T, N, C, T * C,
                       (int64_t)N * C, T * N);
  }
  launch_hook("wino_gemm", 1, s, flop);
  rc = launch_status("wino6_gemm");
  if (rc) return rc;
  gemm_done(s);
  if (f6 == 3) hipLaunchKernelGGL((wino6_output_kernel<2, true>), dim3(grid_of(T * (N / 2))), dim3(256), 0, s, Mt, a, B);
  else if (vw2) hipLaunchKernelGGL(wino6_output_kernel<2>, dim3(grid_of(T * (N / 2))), dim3(256), 0, s, Mt, a, B);
  else hipLaunchKernelGGL(wino6_output_kernel<1>, dim3(grid_of(T * N)), dim3(256), 0, s, Mt, a, B);
  return launch_status("wino6_output");
}

// F(4x4,3x3) when the 4x4 tile grid fits and pis_tune key 11 allows it, else F(2x2,3x3)
int wino_tile(int H, int W) { return (tune_get(PIS_TUNE_WINO_F4) != 0 && H % 4 == 0 && W % 4 == 0) ? 4 : 2; }

bool wino_ok(const IGemmArgs& a) {
  return a.tap_mode == TAP_CONV3 && a.epi == EPI_NHWC && a.H % 2 == 0 && a.W % 2 == 0 && a.Csrc % 4 == 0 &&
         a.N % 4 == 0 && a.lds % 4 == 0 && a.ldd % 4 == 0 && (!(a.flags & PIS_MASK) || a.ldm % 4 == 0);
}

// where launch_wino3x3 keeps V inside its workspace (pis_conv3x3_bwd_prep writes it there)
float* wino_v_slot(void* ws, int C, int N) { return (float*)ws + (size_t)36 * N * C; }

size_t wino_ws_bytes(int B, int H, int W, int C, int N) {
  const int m = wino_tile(H, W), nxi = (m + 2) * (m + 2);
  const int64_t T = (int64_t)B * (H / m) * (W / m);
  // + the fp16x3 tile maxima after M: per (tile, 64-channel chunk) of V (wino_tmax_slot)
  const int64_t extra = T * ((C + 63) / 64) + 8;
  const size_t f4 = (size_t)(nxi * ((int64_t)N * C + T * C + T * N) + extra) * sizeof(float) + 1024;
  return wino6_layer(B, H, W, C, N) ? std::max(f4, wino6_ws_bytes(B, H, W, C, N)) : f4;
}

static int wino_prep_check(const void* ws, int B, int H, int W, int C, int N);

// a describes the direct conv (src/lds = input, wt/ldw = KRSC weights, N outputs, epilogue)
int launch_wino3x3(const IGemmArgs& a, int B, void* ws, hipStream_t s, float* keep_v, bool v_ready) {
  const int C = a.Csrc, N = a.N;
  const int m = wino_tile(a.H, a.W), nxi = (m + 2) * (m + 2);
  const int64_t T = (int64_t)B * (a.H / m) * (a.W / m);
  float* U = (float*)ws;
  float* V = U + (size_t)nxi * N * C;
  float* Mt = V + (size_t)nxi * T * C;
  if (keep_v && m == 4) V = keep_v;
  if (v_ready && m == 4) {
    const int rc = wino_prep_check(ws, B, a.H, a.W, C, N);
    if (rc) return rc;
  }
  // F(6x6,3x3): the deep layers' forward and input gradient (no kept or prepared F(4x4) transforms)
  if (m == 4 && !keep_v && !v_ready && wino6_layer(B, a.H, a.W, C, N) && N % 64 == 0 && C % 32 == 0)
    return launch_wino6(a, B, ws, s);
  const double flop = 2.0 * nxi * (double)T * N * C;
  if (a.filter_ready && m != 4)
    return set_error("launch_wino3x3: PIS_FILTER_READY needs the F(4x4,3x3) GEMM path"), PIS_ERR_ARG;
  if (wino_gemm_out_wanted(m, T, C, N)) {
    // the pre-split filter planes (1.5x U's bytes) go where M would have been
    __bf16* Up = reinterpret_cast<__bf16*>(Mt);
    if (a.filter_ready) Up = const_cast<__bf16*>(reinterpret_cast<const __bf16*>(a.wt));
    else launch_wino4_filter(a, N, C, U, 0, Up, s, wino_gemm_out_h3());
    float* tmax = wino_gemm_out_h3() ? wino_tmax_slot(ws, B, a.H, a.W, C, N) : nullptr;
    if (!v_ready)
      launch_wino4_input(T, C, s, a.src, a.lds, B, a.H, a.W,
                         C, V, tmax);
    int rc = launch_status("wino_transforms");
    if (rc) return rc;
    launch_hook("wino_gemm_out", 0, s, flop);
    rc = launch_wino_gemm_out(V, Up, a, B, T, s, tmax);
    launch_hook("wino_gemm_out", 1, s, flop);
    gemm_done(s);
    return rc;
  }
  if (v_ready && m != 4) return set_error("launch_wino3x3: prepared transforms need F(4x4,3x3)"), PIS_ERR_ARG;
  if (a.w_unflipped && (m != 4 || N % 32 || C % 32))
    return set_error("launch_wino3x3: unflipped weights need F(4x4,3x3) and 32-aligned channels"), PIS_ERR_ARG;
  if (m == 4) {
    if (a.filter_ready) U = const_cast<float*>(a.wt);
    else launch_wino4_filter(a, N, C, U, 0, nullptr, s);
    if (!v_ready) launch_wino4_input(T, C, s, a.src, a.lds, B, a.H, a.W, C, V, nullptr);
  } else {
    hipLaunchKernelGGL(wino_filter_kernel, dim3(grid_of((int64_t)N * C)), dim3(256), 0, s, a.wt, a.ldw, N, C, U);
    hipLaunchKernelGGL(wino_input_kernel, dim3(grid_of(T * (C / 4))), dim3(256), 0, s, a.src, a.lds, B, a.H, a.W,
                       C, V);
  }
  int rc = launch_status("wino_transforms");
  if (rc) return rc;
    launch_hook("wino_gemm", 0, s, flop);
  const int v = tune_get(PIS_TUNE_WINO_TILE);
  if (v == 1 && N % 256 == 0) {
    const dim3 grid((int)cdiv(T, 128) * (N / 256), nxi);
    hipLaunchKernelGGL((gemm_nt_kernel<128, 256>), grid, dim3(256), 0, s, V, U, Mt, (int)T, N, C, T * C,
                       (int64_t)N * C, T * N);
    rc = launch_status("wino_gemm");
  } else if (v == 4 && N % 64 == 0 && C % 32 == 0) {
    // fp16x3 with per-K-step power-of-two tile scales (gemm_nt_h3_bk32_kernel)
    if (N % 128 == 0) {
      const dim3 grid((int)cdiv(T, 128) * (N / 128), nxi);
      hipLaunchKernelGGL((gemm_nt_h3_bk32_kernel<128, 128, 3>), grid, dim3(256), 0, s, V, U, Mt, (int)T, N, C,
                         T * C, (int64_t)N * C, T * N);
    } else {
      const dim3 grid((int)cdiv(T, 128) * (N / 64), nxi);
      hipLaunchKernelGGL((gemm_nt_h3_bk32_kernel<128, 64, 4>), grid, dim3(256), 0, s, V, U, Mt, (int)T, N, C,
                         T * C, (int64_t)N * C, T * N);
    }
    rc = launch_status("wino_gemm");
  } else if (v >= 3 && N % 128 == 0) {
    // K-step 32 single-buffer variant where C allows: 2-9 % faster (tools/bench_gemm.py)
    const dim3 grid((int)cdiv(T, 128) * (N / 128), nxi);
    if (C % 32 == 0)
      hipLaunchKernelGGL((gemm_nt_x6_bk32_kernel<128, 128, 3>), grid, dim3(256), 0, s, V, U, Mt, (int)T, N, C,
                         T * C, (int64_t)N * C, T * N);
    else
      hipLaunchKernelGGL((gemm_nt_x6_kernel<128, 128>), grid, dim3(256), 0, s, V, U, Mt, (int)T, N, C, T * C,
                         (int64_t)N * C, T * N);
    rc = launch_status("wino_gemm");
  } else if (v >= 3 && N % 64 == 0) {
    const dim3 grid((int)cdiv(T, 128) * (N / 64), nxi);
    if (C % 32 == 0)
      hipLaunchKernelGGL((gemm_nt_x6_bk32_kernel<128, 64, 3>), grid, dim3(256), 0, s, V, U, Mt, (int)T, N, C,
                         T * C, (int64_t)N * C, T * N);
    else
      hipLaunchKernelGGL((gemm_nt_x6_kernel<128, 64>), grid, dim3(256), 0, s, V, U, Mt, (int)T, N, C, T * C,
                         (int64_t)N * C, T * N);
    rc = launch_status("wino_gemm");
  } else if (v == 2 && N % 128 == 0) {
    const dim3 grid((int)cdiv(T, 128) * (N / 128), nxi);
    hipLaunchKernelGGL((gemm_nt_kernel<128, 128>), grid, dim3(256), 0, s, V, U, Mt, (int)T, N, C, T * C,
                       (int64_t)N * C, T * N);
    rc = launch_status("wino_gemm");
  } else if (v == 2 && N % 64 == 0) {
    const dim3 grid((int)cdiv(T, 128) * (N / 64), nxi);
    hipLaunchKernelGGL((gemm_nt_kernel<128, 64>), grid, dim3(256), 0, s, V, U, Mt, (int)T, N, C, T * C,
                       (int64_t)N * C, T * N);
    rc = launch_status("wino_gemm");
  } else {
    IGemmArgs gm{};
    gm.src = V; gm.lds = C; gm.Hs = 1; gm.Ws = (int)T; gm.H = 1; gm.W = (int)T; gm.M = (int)T;
    gm.Csrc = C; gm.ntaps = 1; gm.tap_mode = TAP_ONE; gm.wt = U; gm.ldw = C; gm.N = N;
    gm.epi = EPI_NHWC; gm.dst = Mt; gm.ldd = N; gm.flags = 0;
    gm.bs_src = T * C; gm.bs_wt = (int64_t)N * C; gm.bs_dst = T * N;
    rc = launch_igemm(gm, s, nxi);
  }
  launch_hook("wino_gemm", 1, s, flop);
  if (rc) return rc;
  gemm_done(s);
  if (m == 4)
    launch_wino4_output(Mt, a, B, T, N, s);
  else
    hipLaunchKernelGGL(wino_output_kernel, dim3(grid_of(T * (N / 4))), dim3(256), 0, s, Mt, a, B);
  return launch_status("wino_output");
}

// the F(4x4,3x3) filter transform a conv call with these shapes consumes (pis_conv3x3_filter):
// 1 fp32 U[36][N][C] for the batched GEMMs, 2 the bf16x6 planes of the fused 64 -> 64
// contraction, 0 none (not the F(4x4,3x3) GEMM path). C = contraction channels, N = outputs.
int wino_filter_format(int B, int H, int W, int C, int N, bool kept) {
  if (wino_tile(H, W) != 4) return 0;
  const int64_t T = (int64_t)B * (H / 4) * (W / 4);
  if (wino_gemm_out_wanted(4, T, C, N)) return 2;
  return 1;
}

int launch_wino4_filter_only(const float* w, int C, int N, int dgrad, int format, void* out, hipStream_t s) {
  IGemmArgs a{};
  a.wt = w; a.ldw = 9 * C; a.w_unflipped = dgrad;
  if (dgrad && (N % 32 || C % 32)) return set_error("pis_conv3x3_filter: the input-gradient transform needs "
                                                    "32-aligned channels"), PIS_ERR_ARG;
  if (format == 2 && wino_gemm_out_h3() && (C % 64 || N % 4))
    return set_error("pis_conv3x3_filter: fp16x3 planes need 64 x k contraction channels"), PIS_ERR_ARG;
  if (format == 2) launch_wino4_filter(a, N, C, nullptr, 0, reinterpret_cast<__bf16*>(out), s, wino_gemm_out_h3());
  else launch_wino4_filter(a, N, C, reinterpret_cast<float*>(out), 0, nullptr, s);
  return launch_status("wino_filter");
}

// jobs: (w, out, contraction C, outputs N, dgrad, format) — validated by the caller
int launch_wino4_filter_batch(int n, const float* const* w, void* const* out, const int* C, const int* N,
                              const int* dgrad, const int* format, hipStream_t s) {
  if (n <= 0) return PIS_OK;
  if (n > FILTER_MAX_JOBS) return set_error("pis_conv3x3_filters: more than 40 jobs"), PIS_ERR_ARG;
  FilterBatch fb{};
  fb.n = n;
  int total = 0;
  for (int k = 0; k < n; ++k) {
    if (dgrad[k] && (N[k] % 32 || C[k] % 32))
      return set_error("pis_conv3x3_filters: an input-gradient transform needs 32-aligned channels"), PIS_ERR_ARG;
    const int planes = format[k] == 2 ? (wino_gemm_out_h3() ? 2 : 1) : 0;
    if (planes == 2 && (C[k] % 64 || N[k] % 4))
      return set_error("pis_conv3x3_filters: fp16x3 planes need 64 x k contraction channels"), PIS_ERR_ARG;
    const int blocks = planes == 2 ? N[k] / 4 : dgrad[k] ? (N[k] / 32) * (C[k] / 32) : grid_of((int64_t)N[k] * C[k]);
    fb.j[k] = FilterJobDev{w[k], out[k], N[k], C[k], dgrad[k], planes, blocks, format[k] == 4 ? 6 : 4};
    fb.start[k] = total;
    total += blocks;
  }
  fb.start[n] = total;
  hipLaunchKernelGGL(wino4_filter_batch_kernel, dim3(total), dim3(256), 0, s, fb);
  return launch_status("wino_filter_batch");
}

int launch_wino_input(const float* x, int ldx, int B, int H, int W, int C, float* V, hipStream_t s, int m) {
  const int64_t T = (int64_t)B * (H / m) * (W / m);
  if (m == 4)
    launch_wino4_input(T, C, s, x, ldx, B, H, W, C, V);
  else
    hipLaunchKernelGGL(wino_input_kernel, dim3(grid_of(T * (C / 4))), dim3(256), 0, s, x, ldx, B, H, W, C, V);
  return launch_status("wino_input");
}

// channels per thread of the F(3x3,4x4) dz passes (pis_tune key 40): 2 where 256 is a multiple of
// N / 2 (the bias partials' channel-group rule), else 4
// channels per thread of the dz passes: 2 where 256 % (N / 2) == 0 (144-162 registers; the float4
// form, needed for N = 1024, holds 256 + 30 and one wave per SIMD; measured neutral on the step)
static int dz_vw(int N) { return N % 2 == 0 && 256 % (N / 2) == 0 ? 2 : 4; }

// blocks of the F(3x3,4x4) dz pass = rows of its bias partials; dz_bias_rows_max: for any key 40
int wino_dz_blocks(int B, int H, int W, int N, int m) {
  return grid_of((int64_t)B * (H / m) * (W / m) * (N / (m == 4 ? dz_vw(N) : 4)));
}
int wino_dz_blocks_max(int B, int H, int W, int N, int m) {
  return std::max(grid_of((int64_t)B * (H / m) * (W / m) * (N / 4)),
                  m == 4 && N % 2 == 0 ? grid_of((int64_t)B * (H / m) * (W / m) * (N / 2)) : 0);
}

int launch_wino_dz(const float* dz, int ldz, int B, int H, int W, int N, float* E, hipStream_t s, int m,
                   float* bpart) {
  const int64_t T = (int64_t)B * (H / m) * (W / m);
  if (m == 4 && dz_vw(N) == 2)
    hipLaunchKernelGGL(wino4_dz_kernel<2>, dim3(grid_of(T * (N / 2))), dim3(256), 0, s, dz, ldz, B, H, W, N, E, bpart);
  else if (m == 4)
    hipLaunchKernelGGL(wino4_dz_kernel<4>, dim3(grid_of(T * (N / 4))), dim3(256), 0, s, dz, ldz, B, H, W, N, E, bpart);
  else
    hipLaunchKernelGGL(wino_dz_kernel, dim3(grid_of(T * (N / 4))), dim3(256), 0, s, dz, ldz, B, H, W, N, E);
  return launch_status("wino_dz");
}

int launch_wino_dz2(const float* dz, int ldz, int B, int H, int W, int N, float* V, float* E, float* bpart,
                    hipStream_t s, float* tmax) {
  const int64_t T = (int64_t)B * (H / 4) * (W / 4);
  const int vw = dz_vw(N);
  const dim3 grid(grid_of(T * (N / vw)));
  if (tmax && vw == 2)
    hipLaunchKernelGGL((wino4_dz2_kernel<true, 2>), grid, dim3(256), 0, s, dz, ldz, B, H, W, N, V, E, bpart, tmax);
  else if (tmax)
    hipLaunchKernelGGL((wino4_dz2_kernel<true, 4>), grid, dim3(256), 0, s, dz, ldz, B, H, W, N, V, E, bpart, tmax);
  else if (vw == 2)
    hipLaunchKernelGGL((wino4_dz2_kernel<false, 2>), grid, dim3(256), 0, s, dz, ldz, B, H, W, N, V, E, bpart, nullptr);
  else
    hipLaunchKernelGGL((wino4_dz2_kernel<false, 4>), grid, dim3(256), 0, s, dz, ldz, B, H, W, N, V, E, bpart, nullptr);
  return launch_status("wino_dz2");
}

// pis_conv3x3_bwd_prep decides whether its V carries tile maxima (wino_fused_h3_planned) from the
// tune state at ITS call; the dgrad_ex that consumes the V decides again at its own. A changed
// knob in between would make the fused fp16x3 kernel read stale or unwritten scales, so every prep
// is recorded (workspace, shape, decision) and a prepared dgrad must find a matching record.
namespace {
struct PrepRecord {
  const void* ws;
  int B, H, W, C, N;
  bool tmax;
};
thread_local PrepRecord g_prep[16];
thread_local int g_prep_next = 0;
}  // namespace

void wino_prep_record(const void* ws, int B, int H, int W, int C, int N, bool tmax) {
  for (auto& r : g_prep)
    if (r.ws == ws) r.ws = nullptr;  // the workspace's previous content is gone
  g_prep[g_prep_next] = PrepRecord{ws, B, H, W, C, N, tmax};
  g_prep_next = (g_prep_next + 1) % 16;
}

static int wino_prep_check(const void* ws, int B, int H, int W, int C, int N) {
  for (const auto& r : g_prep)
    if (r.ws == ws && r.B == B && r.H == H && r.W == W && r.C == C && r.N == N) {
      if (r.tmax != wino_fused_h3_planned(B, H, W, C, N))
        return set_error("PIS_WINO_PREPARED: pis_conv3x3_bwd_prep wrote %s tile maxima but this call's kernel "
                         "choice needs %s (a pis_tune knob changed in between)",
                         r.tmax ? "" : "no", r.tmax ? "none" : "them"),
               PIS_ERR_ARG;
      return PIS_OK;
    }
  return set_error("PIS_WINO_PREPARED: no pis_conv3x3_bwd_prep of this shape into this workspace"), PIS_ERR_ARG;
}

// where the fp16x3 consumers find the per-(tile, 64-channel chunk) max |V| of their V (after M)
float* wino_tmax_slot(void* ws, int B, int H, int W, int C, int N) {
  const int64_t T = (int64_t)B * (H / 4) * (W / 4);
  return (float*)ws + (size_t)36 * ((int64_t)N * C + T * C + T * N);
}

// the dgrad of these shapes (C contraction = Cout, N = Cin) reads tile maxima (the fused fp16x3
// kernel): its V producer (pis_conv3x3_bwd_prep) must write them
bool wino_fused_h3_planned(int B, int H, int W, int C, int N) {
  if (wino_tile(H, W) != 4) return false;
  const int64_t T = (int64_t)B * (H / 4) * (W / 4);
  return wino_gemm_out_wanted(4, T, C, N) && wino_gemm_out_h3();
}

int launch_wino_wgrad_out(const float* M, int N, int C, float* dw, int accumulate, hipStream_t s, int m,
                          int nsplit, int64_t sstride, WgradOutBias bias) {
  if (bias.rows > 0 && !(m == 4 && ((int64_t)N * C) % 64 == 0))
    return set_error("wino_wgrad_out: the folded bias needs the tiled F(3x3,4x4) transform"), PIS_ERR_ARG;
  const int64_t NC = (int64_t)N * C;
  auto a16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
  if (m == 4 && NC % 64 == 0 && C % 4 == 0 && tune_get(PIS_TUNE_WGRAD_OUT) == 1 && a16(M) && a16(dw) &&
      sstride % 4 == 0) {
    // the widest block that still leaves >= 512 blocks (every CU busy twice)
    const int nb = bias.rows > 0 ? (N + 255) / 256 : 0;
    const int epb = (NC % 256 == 0 && NC / 256 >= 512) ? 256 : (NC % 128 == 0 && NC / 128 >= 512) ? 128 : 64;
    const dim3 grid((unsigned)(NC / epb + nb));
    if (epb == 256)
      hipLaunchKernelGGL(wino4_wgrad_out_v4_kernel<256>, grid, dim3(256), 0, s, M, N, C, dw, accumulate, nsplit,
                         sstride, bias, nb);
    else if (epb == 128)
      hipLaunchKernelGGL(wino4_wgrad_out_v4_kernel<128>, grid, dim3(256), 0, s, M, N, C, dw, accumulate, nsplit,
                         sstride, bias, nb);
    else
      hipLaunchKernelGGL(wino4_wgrad_out_v4_kernel<64>, grid, dim3(256), 0, s, M, N, C, dw, accumulate, nsplit,
                         sstride, bias, nb);
  } else if (m == 4 && ((int64_t)N * C) % 64 == 0) {
    const int nb = bias.rows > 0 ? (N + 255) / 256 : 0;
    hipLaunchKernelGGL(wino4_wgrad_out_tiled_kernel, dim3((unsigned)((int64_t)N * C / 64 + nb)), dim3(256), 0, s, M,
                       N, C, dw, accumulate, nsplit, sstride, bias, nb);
  } else if (m == 4)
    hipLaunchKernelGGL(wino4_wgrad_out_kernel, dim3(grid_of((int64_t)N * C)), dim3(256), 0, s, M, N, C, dw,
                       accumulate, nsplit, sstride);
  else if (nsplit == 1)
    hipLaunchKernelGGL(wino_wgrad_out_kernel, dim3(grid_of((int64_t)N * C)), dim3(256), 0, s, M, N, C, dw,
                       accumulate);
  else
    return set_error("wino_wgrad_out: split slabs need F(3x3,4x4)"), PIS_ERR_ARG;
  return launch_status("wino_wgrad_out");
}

// ---- tooling: time one batched NT GEMM variant (tools/bench_gemm.py) ----------------------
// C[b] (M x N) = A[b] (M x K) . B[b]^T (N x K), batch b over gridDim.y, all row-major fp32.
// variant: 0 bf16x6 128x128, 1 its no-global-load timing twin, 2 its no-split timing twin,
// 3 fp32 MFMA 128x128, 4 bf16x6 128x64, 5/6 the K-step-32 single-buffer bf16x6 128x128 at 2 / 3
// waves per SIMD, 7 its 128x64, 10/11 the fp16x3 128x128 unscaled / scaled, 12 its 128x64, 13 / 14
// the scaled one's no-load / no-staging timing twins (wrong results), 15 the fp16x3 256 x 256 LDS-DMA
// kernel (M, N % 256 == 0), 16 its 4-stage 16-deep ring form.
// Requires N % 128 == 0 (64 for 4, 7, 12), K % 16 == 0 (32 from variant 5).
extern "C" int pis_debug_gemm_nt(const float* A, const float* B, float* C, int M, int N, int K, int batch,
                                 int variant, pis_stream_t stream) {
  const int bn = variant == 4 || variant == 7 || variant == 12 ? 64 : 128;
  PIS_CHECK_ARG(A && B && C && M > 0 && N > 0 && K > 0 && batch > 0 && K % (variant >= 5 ? 32 : 16) == 0 &&
                    N % bn == 0,
                "pis_debug_gemm_nt: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((int)cdiv(M, 128) * (N / bn), batch);
  const int64_t sa = (int64_t)M * K, sb = (int64_t)N * K, sc = (int64_t)M * N;
  switch (variant) {
    case 0: hipLaunchKernelGGL((gemm_nt_x6_kernel<128, 128>), grid, dim3(256), 0, s, A, B, C, M, N, K, sa, sb, sc); break;
    case 1: hipLaunchKernelGGL((gemm_nt_x6_kernel<128, 128, 1>), grid, dim3(256), 0, s, A, B, C, M, N, K, sa, sb, sc); break;
    case 2: hipLaunchKernelGGL((gemm_nt_x6_kernel<128, 128, 2>), grid, dim3(256), 0, s, A, B, C, M, N, K, sa, sb, sc); break;
    case 3: hipLaunchKernelGGL((gemm_nt_kernel<128, 128>), grid, dim3(256), 0, s, A, B, C, M, N, K, sa, sb, sc); break;
    case 4: hipLaunchKernelGGL((gemm_nt_x6_kernel<128, 64>), grid, dim3(256), 0, s, A, B, C, M, N, K, sa, sb, sc); break;
    case 5: hipLaunchKernelGGL((gemm_nt_x6_bk32_kernel<128, 128>), grid, dim3(256), 0, s, A, B, C, M, N, K, sa, sb, sc); break;
    case 6: hipLaunchKernelGGL((gemm_nt_x6_bk32_kernel<128, 128, 3>), grid, dim3(256), 0, s, A, B, C, M, N, K, sa, sb, sc); break;
    case 7: hipLaunchKernelGGL((gemm_nt_x6_bk32_kernel<128, 64, 3>), grid, dim3(256), 0, s, A, B, C, M, N, K, sa, sb, sc); break;
    case 10: hipLaunchKernelGGL((gemm_nt_h3_bk32_kernel<128, 128, 3, false>), grid, dim3(256), 0, s, A, B, C, M, N, K, sa, sb, sc); break;
    case 11: hipLaunchKernelGGL((gemm_nt_h3_bk32_kernel<128, 128, 3>), grid, dim3(256), 0, s, A, B, C, M, N, K, sa, sb, sc); break;
    case 12: hipLaunchKernelGGL((gemm_nt_h3_bk32_kernel<128, 64, 4>), grid, dim3(256), 0, s, A, B, C, M, N, K, sa, sb, sc); break;
    case 13: hipLaunchKernelGGL((gemm_nt_h3_bk32_kernel<128, 128, 3, true, 1>), grid, dim3(256), 0, s, A, B, C, M, N, K, sa, sb, sc); break;
    case 14: hipLaunchKernelGGL((gemm_nt_h3_bk32_kernel<128, 128, 3, true, 2>), grid, dim3(256), 0, s, A, B, C, M, N, K, sa, sb, sc); break;
    default: set_error("pis_debug_gemm_nt: unknown variant %d", variant); return PIS_ERR_ARG;
  }
  return launch_status("debug_gemm_nt");
}

}  // namespace pis
