// Implicit-GEMM argument block shared by the direct (igemm.hip) and Winograd
// (winograd.hip) 3x3-conv paths.
#pragma once
#include "common.h"

namespace pis {

enum TapMode { TAP_CONV3 = 0, TAP_UP2 = 1, TAP_ONE = 2 };
enum EpiMode { EPI_NHWC = 0, EPI_SCATTER2 = 1 };

struct IGemmArgs {
  const float* src;  // NHWC source
  int lds;           // channel stride of src
  int Hs, Ws;        // source spatial dims
  int H, W;          // output pixel grid
  int M;             // B*H*W
  int Csrc;          // channels read per tap
  int ntaps;
  int tap_mode;
  const float* wt;   // Bt[N][ntaps*Csrc]
  int ldw;
  int N;
  // epilogue
  int epi;
  const float* bias;
  const float* scale;  // [B][N]
  const float* mask;   // [M][ldm]
  int ldm;
  float* dst;
  int ldd;
  int flags;
  int cout_t;          // EPI_SCATTER2: n = (i*2+j)*cout_t + o
  float* pool;         // F(4x4,3x3) forward only: also write the 2x2 max pool of dst here ([B][H/2][W/2][N])
  int w_unflipped;     // F(4x4,3x3) input gradient: wt holds the original KRSC weights (no flipped copy)
  int filter_ready;    // F(4x4,3x3): wt holds the layer's filter transform (pis_conv3x3_filter)
  int is_dgrad;        // an input gradient (pis_conv3x3_dgrad*): labels the direct kernel's launch / symbol
  // batched launches (gridDim.y > 1): per-batch element offsets
  int64_t bs_src, bs_wt, bs_dst;
};

// generic implicit GEMM (all tap modes); `batches` independent problems via gridDim.y
int launch_igemm(const IGemmArgs& a, hipStream_t s, int batches = 1);
// 3x3 conv (fwd or dgrad-on-flipped-weights): halo kernel when the grid allows, else igemm
int launch_conv3x3(const IGemmArgs& a, hipStream_t s);
// Winograd F(4x4,3x3) / F(2x2,3x3) path of the same conv (winograd.hip); B = images in a.src
bool wino_ok(const IGemmArgs& a);
// output tile edge of the Winograd fwd/dgrad path for this grid: 4 (F(4x4,3x3)) or 2
int wino_tile(int H, int W);
size_t wino_ws_bytes(int B, int H, int W, int C, int N);
// keep_v (optional, F(4x4) only): V is written there instead of the workspace and left for
// the layer's weight gradient (pis_conv3x3_wgrad_keep)
// v_ready: V (F(4x4) only) is already in the workspace (pis_conv3x3_bwd_prep)
int launch_wino3x3(const IGemmArgs& a, int B, void* ws, hipStream_t s, float* keep_v = nullptr,
                   bool v_ready = false);
float* wino_v_slot(void* ws, int C, int N);
// one pass over dz: V (input-gradient input transform) and E + bias partials (weight gradient)
// (tmax != NULL: also the per-tile max |V| the fused fp16x3 dgrad reads, at wino_tmax_slot)
int launch_wino_dz2(const float* dz, int ldz, int B, int H, int W, int N, float* V, float* E, float* bpart,
                    hipStream_t s, float* tmax = nullptr);
float* wino_tmax_slot(void* ws, int B, int H, int W, int C, int N);
bool wino_fused_h3_planned(int B, int H, int W, int C, int N);
// pis_conv3x3_bwd_prep's record of the V it wrote into ws (checked by the prepared dgrad)
void wino_prep_record(const void* ws, int B, int H, int W, int C, int N, bool tmax);
// does pis_conv3x3_dgrad_ex take F(4x4,3x3) Winograd for this layer with this workspace?
bool dgrad_wino4_planned(int B, int H, int W, int Cin, int Cout, int ldz, size_t ws_bytes);
// Winograd weight-gradient pieces for tile edge m (2: F(3x3,2x2), 4: F(3x3,4x4)), nxi = (m+2)^2:
// V[nxi][T][C] of x, E[nxi][T][N] of dz, dW from M[nxi][N][C]
int launch_wino_input(const float* x, int ldx, int B, int H, int W, int C, float* V, hipStream_t s, int m);
// bpart (m == 4 only, optional, N / 4 must divide 256): per-block channel sums of dz,
// [wino_dz_blocks()][N], for the bias gradient
int launch_wino_dz(const float* dz, int ldz, int B, int H, int W, int N, float* E, hipStream_t s, int m,
                   float* bpart = nullptr);
int wino_dz_blocks(int B, int H, int W, int N, int m);
// F(6x6,3x3) for the forward and input gradient of this layer (pis_tune key 47; symmetric in Cin / Cout)
bool wino6_layer(int B, int H, int W, int Cin, int Cout);
int launch_wino6_filter_only(const float* w, int C, int N, int dgrad, void* out, hipStream_t s);
int wino_dz_blocks_max(int B, int H, int W, int N, int m);  // the largest grid a dz pass of F(m x m) launches (rows of bias partials)
// M: nsplit split-K slabs sstride floats apart, summed in slab order (nsplit > 1 needs m == 4)
// The F(3x3,4x4) weight gradient's bias gradient, folded into its output-transform launch:
// db[n] (+)= scale x sum_{r < rows} part[r][n] (fixed order), part = the GEMM's [split][N] column
// sums of E plane WINO4_BIAS_XI; rows == 0: none
struct WgradOutBias {
  const float* part;
  int rows;
  float* db;
  float scale;
};
// E[7] = E[(1, 1)] = c^2 x (sum of the tile's 16 dz values), c = fp32(1/3) (w4_g4 row 1: the point 1)
constexpr int WINO4_BIAS_XI = 7;
constexpr float WINO4_BIAS_SCALE = (float)(1.0 / ((double)(1.0f / 3.0f) * (double)(1.0f / 3.0f)));
int launch_wino_wgrad_out(const float* M, int N, int C, float* dw, int accumulate, hipStream_t s, int m,
                          int nsplit = 1, int64_t sstride = 0, WgradOutBias bias = WgradOutBias{});

// direct 3x3 conv in fp16x3 (direct.hip): shapes it covers, its workspace (split weights), the
// launch (dgrad_orig: an input gradient whose a.wt holds the ORIGINAL KRSC weights)
bool direct_h3_shape_ok(int H, int W, int C, int N, int ldx);
size_t direct_h3_ws_bytes(int C, int N);
int launch_direct_h3(const IGemmArgs& a, int B, void* ws, size_t ws_bytes, hipStream_t s, bool dgrad_orig,
                     bool ready = false);
int launch_direct_wsplit_batch(int n, const float* const* w, void* const* out, const int* Cin, const int* Cout,
                               const int* dgrad, hipStream_t s);
// pis_tune key 29's policy for a contraction of C channels into N outputs on an H x W grid
bool direct_h3_wanted(int H, int W, int C, int N, int ldx);
// ... and for the layer's weight gradient (the direct fp16x3 wgrad kernel): its workspace, launch
bool direct_w_wanted(int B, int H, int W, int Cin, int Cout, int ldx, int ldz);
size_t direct_w_ws_bytes(int B, int H, int W, int Cin, int Cout);
int launch_direct_wgrad(const float* x, int ldx, const float* dz, int ldz, float* dw, float* db, int B, int H, int W,
                        int Cin, int Cout, int acc, void* ws, size_t ws_bytes, hipStream_t s);

// transposed-conv GEMMs (convt.hip): 0 = launched, 1 = shape not covered, < 0 = error
int launch_convt_gemm(int mode, const float* a, int lda, const float* bt, int B, int h, int w, int cin, int cout,
                      const float* bias, const float* mask, int ldm, float* dst, int ldd, int flags,
                      hipStream_t s);

}  // namespace pis
