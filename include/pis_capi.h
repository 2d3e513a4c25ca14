/*
 * pis_capi.h — C-ABI of the MI355X (gfx950) training-step kernels for the
 * PDE-constrained U-Net (seemapoudel58/Physics_informed_image_segmentation).
 *
 * The reference is pure Python/PyTorch: its "operator API" is the module
 * surface of src/unet.py, src/pde.py, src/loss.py, src/metrics.py and the step
 * loop of src/train.py. Every entry point below replaces the ATen op(s) the
 * reference reaches at the cited line; the Python mirror of the reference
 * interface (physics_informed_image_segmentation_amd/) binds them with ctypes
 * (INTEGRATION.md).
 *
 * Conventions
 *  - Activations are pixel-major NHWC fp32. "ld*" is the channel stride of a
 *    tensor (elements between consecutive pixels), so a producer can write
 *    straight into a channel slice of a concat buffer (src/unet.py:190-202).
 *  - Conv weights are KRSC ([Cout][3][3][Cin]) = the physical layout of an
 *    OIHW channels_last parameter; ConvTranspose weights are stored
 *    [2][2][Cout][Cin] (logical (Cin, Cout, 2, 2), state_dict compatible).
 *  - The caller owns every buffer (workspace included); nothing allocates,
 *    nothing synchronises; kernels are launched on `stream` (a hipStream_t).
 *  - Return 0 on success, a negative PIS_ERR_* otherwise; the message is in
 *    pis_last_error() (thread-local). No C++ exception crosses the ABI.
 */
#ifndef PIS_CAPI_H
#define PIS_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* pis_stream_t; /* hipStream_t */

#define PIS_OK 0
#define PIS_ERR_ARG (-1)
#define PIS_ERR_LAUNCH (-2)
#define PIS_ERR_WORKSPACE (-3)

/* epilogue / behaviour flags */
#define PIS_RELU 1       /* y = max(y, 0)                                     */
#define PIS_SCALE 2      /* y *= scale[b*C + c]  (Dropout2d keep-scale)       */
#define PIS_MASK 4       /* y *= (mask[pix*ldm + c] > 0)  (ReLU backward)     */
#define PIS_ACCUMULATE 8 /* dst += result instead of dst = result             */
#define PIS_WINO_PREPARED 16 /* conv3x3 dgrad_ex / wgrad_keep: pis_conv3x3_bwd_prep already wrote this
                                layer's dz transforms into the call's workspace          */
#define PIS_W_UNFLIPPED 32   /* conv3x3 dgrad_ex with PIS_WINO_PREPARED: w_flip is the layer's ORIGINAL
                                KRSC weight (the F(4x4) filter transform rotates it in place) */
#define PIS_FILTER_READY 64  /* conv3x3 fwd_ex / fwd_keep / fwd_pool / dgrad_ex: the weight argument is
                                the layer's filter transform from pis_conv3x3_filter (same shape and
                                direction), so the call launches no filter transform of its own */

const char* pis_last_error(void);
int pis_version(void);

/* Kernel-variant knobs (process-wide). value < 0 queries; returns the previous
 * value or PIS_ERR_ARG. Defaults are the measured best on MI355X.            */
#define PIS_TUNE_IGEMM_BK 1 /* implicit-GEMM K-step: 16 or 32 */
#define PIS_TUNE_DEBUG_NOLOAD 2 /* timing only: implicit GEMM skips its global loads (wrong results) */
#define PIS_TUNE_CONV_HALO 3 /* 1: 3x3 conv fwd/dgrad from a staged input halo (W%16==0, H%8==0) */
#define PIS_TUNE_HALO_VARIANT 4 /* 0: auto, 1: 4-channel slices for BN=64, 2: BN=256 tiles when N >= 256, 3: 8-channel slices for BN=64 */
#define PIS_TUNE_WGRAD_VARIANT 5 /* 0: one 16-pixel segment per stage, 1: two (default) */
#define PIS_TUNE_WGRAD_BLOCKS 6  /* target workgroups of the split-K halo wgrad (default 512: one round at 2 per CU) */
#define PIS_TUNE_C1_WGRAD 7      /* Cin == 1 weight gradient: 0 VALU stream kernel (default), 1 padded MFMA tile */
#define PIS_TUNE_WINOGRAD 8      /* 3x3 convs: 0 direct only; 1 (default) Winograd for fwd/dgrad (*_ex) with >= 256
                                    contraction and >= 128 output channels, for wgrad with >= 128 in and out;
                                    2 Winograd whenever legal */
#define PIS_TUNE_WINO_WGRAD_BLOCKS 9 /* target workgroups of the batched Winograd weight-gradient GEMMs (default 1024;
                                        2048 until round 3: the C2 step 0.6 % slower, profiles/r3_q33_ab_wgrad_blocks.txt) */
#define PIS_TUNE_WINO_TILE 10    /* Winograd batched GEMM: 0 generic igemm, 1 lean NT GEMM 128x256 (N % 256 == 0), 2 lean NT GEMM
                                    128x128|64 on fp32 MFMA, 3 the same at fp32 accuracy on bf16 MFMA ("bf16x6": exact
                                    3-way bf16 split of each operand, the six partial products >= 2^-24), 4 (default)
                                    "fp16x3" on fp16 MFMA: each K-step's operand tiles scaled by a power of two into
                                    fp16 range, split into hi + lo fp16 (22 significant bits), the three products
                                    above 2^-22 accumulated in fp32 (measured error below fp32 MFMA's and bf16x6's) */
#define PIS_TUNE_WINO_F4 11      /* Winograd tile: 0 F(2x2,3x3) fwd/dgrad + F(3x3,2x2) wgrad; 1 (default) F(4x4,3x3) +
                                    F(3x3,4x4) when H % 4 == W % 4 == 0 */
#define PIS_TUNE_WINO_FUSED 12   /* retired (round 3): the one-kernel F(4x4,3x3) was slower than the 3-pass pipeline
                                    on every layer; the key is accepted and ignored */
#define PIS_TUNE_CONVT_GEMM 13   /* transposed conv fwd/dgrad: lean NT GEMM with gather/scatter addressing when
                                    Cin, Cout % 16 == 0 — 4 (default) fp16x3, K-step 32 with the loads two K-steps
                                    ahead, epilogue through LDS (16-B pixel stores), and the weight gradient on the
                                    row-staged split-K kernel where Cin >= 256 (needs M, N % 128, w % 32; else 3);
                                    3 fp32-class fp16x3 on fp16 MFMA, K-step 16 (per-wave, per-K-step power-of-two
                                    scales), 1 bf16x6 on bf16 MFMA, 2 on fp32 MFMA; 0 generic implicit GEMM */
#define PIS_TUNE_WGRAD_X6 14     /* Winograd and transposed-conv weight-gradient GEMMs: 3 (default) fp16x3 where the
                                    layer has >= 256 input channels, bf16x6 elsewhere; 1 fp32-accurate bf16x6 on
                                    bf16 MFMA everywhere, 2 fp16x3 (as key 10 = 4) everywhere (-1 % on the step: the
                                    512^2 layers are HBM-bound), 0 fp32 MFMA */
#define PIS_TUNE_WINO_GEMM_OUT 15 /* F(4x4,3x3) 64 -> 64 channels: 1 (default) the 36 bf16x6 contractions fused with
                                     the output transform (M stays on chip; 4 groups of 32 tiles per block), 2 / 3 / 4
                                     the same with 1 / 2 / 8 groups per block (bitwise equal), 0 separate GEMM +
                                     output transform */
#define PIS_TUNE_WINO_DZ2 16     /* pis_conv3x3_bwd_prep: 1 (default) one pass over dz for both transforms, 0 off */
#define PIS_TUNE_WINO_VW 17      /* F(4x4) input / output transforms: 2 (default: half the registers, +2-11 % on the
                                    512^2-256^2 layers) or 4 channels per thread */
#define PIS_TUNE_LOSS_ROWS 18     /* pis_loss_fwd with W % 4 == 0: 1 (default) whole-row bands, 0 16x128 tiles;
                                    both followed by the one-block fixed-order finalize (deterministic) */
#define PIS_TUNE_LOSS_ROWMUL 19  /* whole-row loss forward: rows per block multiplier (1 default: about 1024 blocks;
                                    2, 4: fewer blocks, more row batches per thread) */
#define PIS_TUNE_SLAB_CHUNKS 20  /* thousands of partial slabs over <= 1024 columns (bias gradients): 1 (default)
                                    two-pass chunked row reduction, 0 one column per block. Applies to
                                    reduce_slabs and weights-only reduce_slabs2 calls; a weights + bias
                                    pair is always one merged single-pass launch (csrc/wgrad.hip) */
#define PIS_TUNE_WGRAD_PAIR 21   /* bf16x6 weight-gradient GEMM, 64-wide operand tiles: 0 (default) one 4-pixel run per
                                    lane (2-way conflicted ds_write_b64), 1 lane pairs stage the two 8-B halves of one 16-B
                                    chunk (conflict-free; the two 128-B pixel rows per load cost more: enc1.conv1 -4 %, up1
                                    +9 %, step -0.4 %) */
#define PIS_TUNE_WINO_GEMM_OUT_H3 22 /* the fused 64 -> 64 kernel (key 15): 1 fp16x3 (per-(tile, xi, K-step) power-of-two
                                        scales, hi + lo fp16, 3 products; its filter planes, also those written by
                                        pis_conv3x3_filter(s), switch format with it), 0 bf16x6 */
#define PIS_TUNE_WINO_H3_PRE 23  /* retired (round 3): producer-written row scales for the batched fp16x3 GEMM measured
                                    slower (GEMM +10 %, input transform +11 %, profiles/r2_q65_*); ignored */
#define PIS_TUNE_WINO_PERSIST 24 /* retired (round 3): the persistent batched GEMM was within +-1 % per layer and
                                    +0.4 % on the step (profiles/r2_q70_*, r2_q72_*); ignored */
#define PIS_TUNE_FUSED_STAGGER 25 /* fused 64 -> 64 kernel in fp16x3 (key 22): 1 the SIMD-partner waves fold one xi late
                                     (stagger; bit-for-bit the same), 0 (default) all waves in lockstep */
#define PIS_TUNE_FUSED_WIDE 26   /* v: the fused contraction + output transform (key 15) for up to 64 x 2^v output
                                    channels (N / 64 blocks per tile group, V re-read from L2, M never written):
                                    2 (default, N <= 256; enc3.conv0 forward -9 %), 1 (N <= 128: enc2.conv0 forward
                                    -21 %, dec1.conv0 input gradient -20 %), 0: 64 outputs only */
#define PIS_TUNE_FUSED_K128 27   /* 1 (default): the fused contraction + output transform also for 128-channel
                                    contractions (128 -> 64, and 128 -> 128 with key 26; the SIMD-partner waves always
                                    staggered: dec1.conv0 forward -11 %, enc2.conv0 input gradient -15 %);
                                    0: 64-channel contractions only */
#define PIS_TUNE_FUSED_PAIR 28   /* retired (round 3): two xi per barrier in the fused kernel was not faster; ignored */
#define PIS_TUNE_DIRECT_H3 29   /* direct 3x3 conv in fp16x3 (csrc/direct.hip; forward, input and weight gradient):
                                   0 off (Winograd / halo kernels), 1 (default) auto: the shallow layers (<= 128
                                   channels on both sides, H >= 256),
                                   2 every shape it covers (H % 8, W % 32, C % 16, N % 64 == 0),
                                   3 auto + the 128 <-> 256-channel layers at 256^2 and 128^2, 4 H >= 128 and
                                   <= 256 channels, 5 H >= 128 (3/4/5 measured slower on the C2 step:
                                   profiles/r3_q8_direct_policy.txt) */
#define PIS_TUNE_DIRECT_WG 30    /* retired (round 3): the double-buffered direct weight gradient (2-row tiles, 512
                                    registers per lane) measured slower than the single-buffer kernel, an eight-wave
                                    form neutral (profiles/r3_q19_wg8.txt); ignored */
#define PIS_TUNE_WGRAD_T 31      /* fp16x3 weight-gradient GEMM (key 14) on plain 128 x 128 tiles (the Winograd weight
                                    gradient): 1 operands staged as stored (float4 rows, transposed LDS reads, 32-pixel
                                    K-steps, block-wide scales), 0 the column-staged wgrad_h3_kernel */
#define PIS_TUNE_DIRECT_PIPE 32  /* direct fp16x3 input gradient (key 29): 1 (default) the epilogue's ReLU-mask rows
                                    loaded during the last chunk's MFMAs (enc1.conv1 -12 %), 0 in the epilogue */
#define PIS_TUNE_DIRECT_W8 33    /* retired (round 3): an 8-wave two-stage direct forward / input gradient (16-row tiles,
                                    one block per CU, next chunk's weights by LDS-DMA and its halo split while this
                                    chunk multiplies) measured 3-14 % slower than the 4-wave kernel
                                    (profiles/r3_q26_direct_w8.txt); ignored */
#define PIS_TUNE_DIRECT_WSTRIP 34 /* retired (round 5): the 2-row strip, LDS-ring and software-pipelined direct weight
                                     gradients measured 1.6-1.8 % slower on the C2 step than the 4-row kernel
                                     (profiles/r4_a_*, r4_b_ab_wblk.txt, r4_k_*); removed, the key is ignored */
#define PIS_TUNE_DIRECT_WBLOCKS 35 /* retired (round 5) with key 34; ignored */
#define PIS_TUNE_HEAD_LOSS_ROWS 36 /* pis_head_loss_fwd: image rows per block (0, default: 4096 / W, at most 16,
                                       doubled while the row bands exceed 2048; 8 at C2 measured 131 us against
                                       134-145 at 16, profiles/r4_ah_head_loss_rows.txt) */
#define PIS_TUNE_DIRECT_WGRAD_ALL 37 /* retired (round 5): the strip weight gradient on every layer was 6.3 % slower
                                        (profiles/r4_a_bench_k37_1.json); ignored */
#define PIS_TUNE_HEAD_LOSS_WIDE 38 /* pis_head_loss_fwd with W % 512 == 0: 1 (default) 1024-thread blocks (16 waves,
                                       one staged row per chunk), 2 the same with three register sets in flight
                                       (measured equal, profiles/r4_q_head_loss_fwd.txt), 0 the 256-thread form */
#define PIS_TUNE_WGRAD_T_DEPTH 39 /* retired (round 5): a third register set in wgrad_h3t_kernel was neutral
                                      (profiles/r4_f_ab.txt); two sets always; ignored */
#define PIS_TUNE_DZ_VW 40 /* retired (round 5): the dz passes take 2 channels per thread wherever 256 % (N / 2) == 0
                               (4 otherwise; the choice measured neutral, profiles/r4_g_ab.txt); ignored */
#define PIS_TUNE_GEMM_256 41 /* retired (round 5): the 256 x 256 LDS-DMA fp16x3 GEMMs measured 25-40 % slower per GEMM
                                  (profiles/r4_i_gemm_256.txt, r4_j_gemm_256_ring.txt); removed; ignored */
#define PIS_TUNE_LAST_WGRAD_MAIN 42 /* host schedule (physics_informed_image_segmentation_amd/unet.py): 1 (default) the
                                         step's last weight gradient (enc1.conv0) on the main stream, idle after
                                         enc1.conv1's input gradient, beside the side stream's enc1.conv1 weight
                                         gradient; 0 on the side stream after it (measured neutral: 22.67 vs
                                         22.66 ms, profiles/r4_l_ab_sched.txt) */
#define PIS_TUNE_DIRECT_W_VWALK 43 /* the 4-row direct weight gradient (key 34 = 0): 1 (default) each block walks a
                                        contiguous run of tiles down the image columns (vertical neighbours share
                                        two x halo rows: L2 hits) with the pairs of one split on one XCD; 0 the
                                        round-3 strided tile order. HBM reads per launch 2218 -> 1674 MB on
                                        dec1.conv0 (1.38x -> 1.04x algorithmic; enc1.conv1 1.03x either way,
                                        profiles/r4_o_direct_wgrad_traffic.txt), time unchanged (r4_n) */
#define PIS_TUNE_DIRECT_WGRAD_MAIN 44 /* retired as a tune key (ignored): the choice moved to the host schedule's
                                           PIS_DIRECT_WGRAD_MAIN environment variable (unet.py), whose default
                                           since round 5 is 1 = direct weight gradients on the main stream, the
                                           side stream ordered after them before its next weight gradient or
                                           bucket all-reduce */
#define PIS_TUNE_GEMM_PRIO 45 /* retired (round 5): s_setprio in the Winograd GEMM was neutral
                                   (profiles/r4_s_ab_gemm_prio.txt); ignored */
#define PIS_TUNE_WINO_OUT_MPF 46 /* Winograd output transform of a masked input gradient: 1 (default) the tile's
                                      ReLU-mask rows loaded with its M values (one memory round trip per tile,
                                      151 VGPRs); 0 in the epilogue. Step 22.25 -> 22.04 ms on one box, 22.43 ->
                                      22.39 on another (profiles/r4_t_ab_wino_out_mpf.txt, r4_u_*): 0.2-0.9 % */
#define PIS_TUNE_WINO_F6 47 /* Winograd F(6x6,3x3) for the forward and input gradient of the deep layers whose
                               contractions run the batched fp16x3 GEMM both ways (csrc/winograd.hip
                               wino6_layer: 64-aligned channels, neither direct nor fused, >= 10 % fewer
                               products than F(4x4) on the ragged 6 x 6 tile grid — 128^2 and 64^2 at C2;
                               their weight gradients keep F(3x3,4x4) with their own transforms): 0
                               (default) F(4x4,3x3) with the kept / prepared transforms; 1 F(6x6), one
                               channel per thread in the transforms; 2 two channels; 3 two channels with
                               runtime-looped (lower-register) transforms. Measured slower on the C2 step
                               (358.7 vs 366.8 img/s, profiles/r6_f6*): the GEMMs -12 % per F(6x6)
                               launch but the 64-value transforms run at ~0.65 of F(4x4)'s bytes/s and
                               the weight gradients' own transforms load the side stream */
#define PIS_TUNE_WGRAD_OUT 48 /* the F(3x3,4x4) weight gradient's slab sum + output transform
                                 (csrc/winograd.hip launch_wino_wgrad_out): 0 64 entries per block, one
                                 float per lane per slab row; 1 (default) float4 lanes, 64-256 entries
                                 per block (bitwise equal: same sums in the same order) */
#define PIS_TUNE_DIRECT_W_ROWS 49 /* the direct weight gradient's tile rows (csrc/direct.hip): 2 (default) two
                                     blocks per CU (51 KB LDS, <= 256 registers each), no register prefetch;
                                     4 (any other value) one block per CU, the next tile's loads in registers.
                                     2 vs 4: -2..-10 % per layer isolated, step 22.08 -> 21.76 ms
                                     (profiles/r6_d1_direct_wgrad_rows.txt) */
#define PIS_TUNE_NKEYS 50
#define PIS_DEBUG_NOLOAD (1 << 16)
int pis_tune(int key, int value);
/* Tooling (tools/bench_gemm.py): time one batched NT GEMM kernel variant in isolation,
 * C[b] = A[b] . B[b]^T row-major fp32 — 0 bf16x6 128x128 (the Winograd GEMM), 1/2 its
 * no-global-load / no-split timing twins (wrong results), 3 fp32 MFMA, 4 bf16x6 128x64, 5/6 the
 * K-step-32 single-LDS-buffer bf16x6 128x128 (2 / 3 waves per SIMD), 7 its 128x64, 10 / 11 the
 * fp16x3 128x128 GEMM unscaled / with per-K-step scales (11 is the Winograd default), 12 its 128x64,
 * 13 / 14 11's no-global-load / no-staging timing twins (wrong results).
 * 5-12 need K % 32 == 0. */
int pis_debug_gemm_nt(const float* A, const float* B, float* C, int M, int N, int K, int batch, int variant,
                      pis_stream_t stream);
/* Tooling (bench.py roofline_loss): one float4 grid-stride launch over n floats of a and b — dst = a + b
 * when dst is given (12 B per element), else a read reduced to one partial per block (8 B per element):
 * the floor any kernel moving the loss's bytes meets at the same size and cache state. */
int pis_debug_stream_probe(const float* a, const float* b, float* dst, int64_t n, float* partial, int grid,
                           pis_stream_t stream);

/* Tooling (tools/bench_head_loss.py --probe): read n floats (n % 4096 == 0) in 16-KB chunks with 1024-thread
 * blocks, eight chunks in flight per lane: mode 0 grid-stride sweep (concurrent reads in one window),
 * mode 1 one contiguous run per block (the row-band kernels' order); partial[grid * 16] wave sums. */
int pis_debug_band_probe(const float* a, int64_t n, int mode, float* partial, int grid, pis_stream_t stream);

/* Scheduling aid: arm an event (hipEvent_t) that the next F(4x4,3x3) convolution launched on this
 * thread (pis_conv3x3_fwd_ex / _dgrad_ex / _fwd_keep / _fwd_pool) records on its stream right after
 * its 36 contractions, before the output transform; the slot then disarms. Lets a caller start
 * MFMA-bound work on another stream while the HBM-bound output transform runs. Returns 1 when
 * the previously armed event was never recorded (NULL disarms), else 0. */
int pis_arm_gemm_event(void* event);

/* Owned HIP streams (hipStreamNonBlocking, the given priority: 0 normal, -1 high). torch's
 * torch.cuda.Stream() hands out a fixed round-robin pool, so a stream that took part in a HIP graph
 * capture is later handed to unrelated code; the engine's weight-gradient stream and the capture
 * stream of a graphed step are owned instead (wrapped with torch.cuda.ExternalStream) and recycled
 * among owners (the Python side never destroys one: PyTorch keeps raw stream handles in autograd
 * nodes and allocator blocks). pis_stream_capture_status: hipStreamCaptureStatus (0 none, 1 active,
 * 2 invalidated) or a negative error. */
int pis_stream_create(int priority, pis_stream_t* out);
/* pis_stream_destroy: for hosts that own their streams' lifetime; the Python host never calls it (its
 * owned streams are recycled, never destroyed: PyTorch keeps raw stream handles beyond their users). */
int pis_stream_destroy(pis_stream_t stream);
int pis_stream_capture_status(pis_stream_t stream);

/* Profiling hook: called on the launching thread right before (phase 0) and after (phase 1)
 * the enqueue of each heavy kernel ("conv3x3_halo", "wino_gemm", "wino_gemm_out", "wgrad3x3_halo",
 * "wino_wgrad_gemm", "direct_h3_fwd", "direct_h3_pool", "direct_h3_dgrad", "direct_wgrad_h3"), with
 * its stream and the MFMA FLOPs it executes ("head_loss_fwd": its algorithmic HBM bytes instead), so
 * a profiler can record HIP events on that stream around exactly that kernel. NULL removes it. */
typedef void (*pis_launch_hook_t)(const char* kernel, int phase, pis_stream_t stream, double flop,
                                  void* user);
void pis_set_launch_hook(pis_launch_hook_t fn, void* user);

/* ---- 3x3 convolution, padding 1, stride 1 (src/unet.py:29,38 nn.Conv2d) ----
 * fwd:  y[p][n] = epi(bias[n] + sum_{r,s,c} x[p+(r-1,s-1)][c] * w[n][r][s][c])
 *       flags: PIS_RELU, PIS_SCALE (scale is [B][Cout]).   Cin==1 or Cin%4==0. */
int pis_conv3x3_fwd(const float* x, int ldx, const float* w_krsc, const float* bias,
                    const float* scale, float* y, int ldy, int B, int H, int W, int Cin,
                    int Cout, int flags, pis_stream_t stream);
/* Same contraction as pis_conv3x3_fwd / pis_conv3x3_dgrad, with a workspace that admits the fast
 * paths: the direct fp16x3 kernel (csrc/direct.hip) on the shallow layers (<= 128 channels both
 * sides, H >= 256; pis_tune key 29), else Winograd F(4x4,3x3) (4x fewer MFMA FLOPs: filter, input
 * and output transforms around 36 batched fp16x3 GEMMs, or the fused contraction + output transform
 * for 64 / 128-channel contractions; F(2x2,3x3) only behind pis_tune(11, 0) or for grids not
 * divisible by 4). ws may be NULL (the fp32-MFMA halo / implicit-GEMM kernels). */
size_t pis_conv3x3_ex_ws(int B, int H, int W, int Cin, int Cout);
int pis_conv3x3_fwd_ex(const float* x, int ldx, const float* w_krsc, const float* bias,
                       const float* scale, float* y, int ldy, int B, int H, int W, int Cin, int Cout,
                       int flags, void* ws, size_t ws_bytes, pis_stream_t stream);
/* w_flip[c][r][s][n] = w[n][2-r][2-s][c]  (dgrad operand, rebuilt each step) */
int pis_conv3x3_flip(const float* w_krsc, float* w_flip, int Cin, int Cout, pis_stream_t stream);
/* dgrad: dx[p][c] = epi(sum_{r,s,n} dz[p+(r-1,s-1)][n] * w_flip[c][r][s][n])
 *        flags: PIS_MASK (mask = this conv's input x), PIS_SCALE ([B][Cin]). */
int pis_conv3x3_dgrad(const float* dz, int ldz, const float* w_flip, const float* mask, int ldm,
                      const float* scale, float* dx, int lddx, int B, int H, int W, int Cin,
                      int Cout, int flags, pis_stream_t stream);
int pis_conv3x3_dgrad_ex(const float* dz, int ldz, const float* w_flip, const float* mask, int ldm,
                         const float* scale, float* dx, int lddx, int B, int H, int W, int Cin,
                         int Cout, int flags, void* ws, size_t ws_bytes, pis_stream_t stream);
/* wgrad: dw[n][r][s][c] (+)= sum_p dz[p][n] x[p+(r-1,s-1)][c];  db[n] (+)= sum_p dz[p][n]
 *        (db may be NULL). flags: PIS_ACCUMULATE. */
/* Kept input transform (training forward -> weight gradient of the same layer): where the
 * forward runs Winograd F(4x4,3x3) and the weight gradient F(3x3,4x4), both transform the
 * same input x with the same B^T; pis_conv3x3_fwd_keep leaves that transform in `keep`
 * (pis_conv3x3_keep_bytes(), 0 = nothing to keep) and pis_conv3x3_wgrad_keep reads it instead
 * of recomputing it. x must be unchanged in between. keep == NULL: plain _ex / wgrad. */
size_t pis_conv3x3_keep_bytes(int B, int H, int W, int Cin, int Cout);
int pis_conv3x3_fwd_keep(const float* x, int ldx, const float* w_krsc, const float* bias,
                         const float* scale, float* y, int ldy, int B, int H, int W, int Cin, int Cout,
                         int flags, void* ws, size_t ws_bytes, float* keep, pis_stream_t stream);
/* The encoder's conv1 + MaxPool2d(2,2) (src/unet.py:126, :177-188): as pis_conv3x3_fwd_keep, and
 * pool[b][h/2][w/2][c] (ld = Cout) = the 2x2 max of the y it wrote — in the F(4x4,3x3) output
 * epilogue when that path runs (no second read of y), else by pis_maxpool2x2_fwd. H, W even; no
 * PIS_ACCUMULATE. */
int pis_conv3x3_fwd_pool(const float* x, int ldx, const float* w_krsc, const float* bias, const float* scale,
                         float* y, int ldy, int B, int H, int W, int Cin, int Cout, int flags, void* ws,
                         size_t ws_bytes, float* keep, float* pool, pis_stream_t stream);
int pis_conv3x3_wgrad_keep(const float* x, int ldx, const float* dz, int ldz, float* dw_krsc, float* db,
                           int B, int H, int W, int Cin, int Cout, int flags, void* ws, size_t ws_bytes,
                           const float* keep, pis_stream_t stream);
/* One pass over a layer's dz for both backward products (no reference counterpart: the two
 * reads of dz that conv2d's input- and weight-gradient make): writes the F(4x4,3x3) input
 * transform into ws_dgrad (for pis_conv3x3_dgrad_ex) and the F(3x3,4x4) dz transform + bias
 * partials into ws_wgrad (for pis_conv3x3_wgrad_keep); both calls then pass PIS_WINO_PREPARED.
 * Returns 1 when done, 0 when this layer / workspace does not take that path (call without the
 * flag), < 0 on error. ws_wgrad must stay untouched until its pis_conv3x3_wgrad_keep ran. */
/* The F(4x4,3x3) filter transform of a conv3x3 layer, ahead of its convolution call (so it can run
 * on another stream, off the critical path). dgrad = 0: for the forward, w = KRSC [Cout][9][Cin];
 * dgrad = 1: for the input gradient, w = the ORIGINAL KRSC weights (rotated in place, as
 * PIS_W_UNFLIPPED). The output format is the one the call with these shapes will consume (fp32
 * U[36][N][C] for the batched GEMMs (followed, with pis_tune(23, 1) and C, N % 64 == 0, by its
 * per-(output, 32-channel chunk) maxima umax[N][C / 32]); for the fused 64->64 contraction the fp16x3 hi / lo planes +
 * one inverse scale per output channel, or with pis_tune(22, 0) the bf16x6 planes: the tune key
 * must not change between this call and the conv call that consumes it); where the call takes the
 * direct fp16x3 kernel (pis_tune key 29) its weight split: fp16 hi / lo planes in the kernel's LDS
 * image + one inverse scale per output channel.
 * pis_conv3x3_filter_bytes returns its size, 0 when that call would take neither the F(4x4,3x3)
 * GEMM path nor the direct kernel (then PIS_FILTER_READY must not be used). Pass the result as the
 * weight argument with PIS_FILTER_READY (dgrad: with PIS_WINO_PREPARED | PIS_W_UNFLIPPED semantics
 * kept). pis_conv3x3_filters: the Winograd transforms in one launch, the direct splits in a second. */
size_t pis_conv3x3_filter_bytes(int B, int H, int W, int Cin, int Cout, int dgrad);
int pis_conv3x3_filter(const float* w, int B, int H, int W, int Cin, int Cout, int dgrad, void* out,
                       size_t out_bytes, pis_stream_t stream);
/* Several layers' filter transforms (as pis_conv3x3_filter) in ONE launch: a layer's own grid is
 * small and latency-bound, here all jobs' blocks run side by side. At most PIS_FILTER_MAX_JOBS. */
typedef struct pis_filter_job {
  const float* w;
  void* out;
  size_t out_bytes;
  int B, H, W, Cin, Cout, dgrad;
} pis_filter_job;
#define PIS_FILTER_MAX_JOBS 40
/* The filter operand format pis_conv3x3_filter(s) would write for these shapes (0 none, 1 F(4x4) U[36][N][C]
 * fp32, 2 the fused kernel's planes, 3 the direct kernel's weight split, 4 F(6x6) U[64][N][C] fp32). */
int pis_conv3x3_filter_format(int B, int H, int W, int Cin, int Cout, int dgrad);
int pis_conv3x3_filters(const pis_filter_job* jobs, int n, pis_stream_t stream);
/* 1 when pis_conv3x3_dgrad_ex of these shapes (and workspace) runs the direct fp16x3 kernel
 * (pis_tune key 29), which accepts PIS_W_UNFLIPPED (the original weights) without
 * PIS_WINO_PREPARED; 0 otherwise. */
int pis_conv3x3_dgrad_direct(int B, int H, int W, int Cin, int Cout, int ldz, size_t ws_bytes);
int pis_conv3x3_bwd_prep(const float* dz, int ldz, int B, int H, int W, int Cin, int Cout, void* ws_dgrad,
                         size_t ws_dgrad_bytes, void* ws_wgrad, size_t ws_wgrad_bytes, pis_stream_t stream);
size_t pis_conv3x3_wgrad_ws(int B, int H, int W, int Cin, int Cout);
int pis_conv3x3_wgrad(const float* x, int ldx, const float* dz, int ldz, float* dw_krsc, float* db,
                      int B, int H, int W, int Cin, int Cout, int flags, void* ws, size_t ws_bytes,
                      pis_stream_t stream);

/* ---- 2x2 stride-2 transposed convolution (src/unet.py:132-153) ----
 * H, W are the INPUT resolution; the output is 2H x 2W.
 * fwd: y[(2h+i,2w+j)][o] = bias[o] + sum_c x[(h,w)][c] * w[i][j][o][c]          */
int pis_convt2x2_fwd(const float* x, int ldx, const float* w_ijoc, const float* bias, float* y,
                     int ldy, int B, int H, int W, int Cin, int Cout, pis_stream_t stream);
/* w_cijo[c][i][j][o] = w_ijoc[i][j][o][c]  (dgrad operand) */
int pis_convt2x2_prep(const float* w_ijoc, float* w_cijo, int Cin, int Cout, pis_stream_t stream);
/* dgrad: dx[(h,w)][c] = epi(sum_{i,j,o} dy[(2h+i,2w+j)][o] * w[i][j][o][c]); flags: PIS_MASK */
int pis_convt2x2_dgrad(const float* dy, int lddy, const float* w_cijo, const float* mask, int ldm,
                       float* dx, int lddx, int B, int H, int W, int Cin, int Cout, int flags,
                       pis_stream_t stream);
/* wgrad: dw[i][j][o][c] (+)= sum_(h,w) dy[(2h+i,2w+j)][o] x[(h,w)][c]; db[o] (+)= sum dy[.][o] */
size_t pis_convt2x2_wgrad_ws(int B, int H, int W, int Cin, int Cout);
int pis_convt2x2_wgrad(const float* x, int ldx, const float* dy, int lddy, float* dw_ijoc,
                       float* db, int B, int H, int W, int Cin, int Cout, int flags, void* ws,
                       size_t ws_bytes, pis_stream_t stream);

/* ---- 2x2 max pooling (src/unet.py:126,181-186) ----
 * H, W are the INPUT resolution. y is contiguous (ld = C).
 * bwd (fused with the skip-gradient sum and the ReLU backward of the pooled
 * block's output):  dx[p][c] = (dskip[p][c] + [p = argmax] dy[q][c]) * (x[p][c] > 0)
 * dskip may be NULL; dx has ld = lddx.                                            */
int pis_maxpool2x2_fwd(const float* x, int ldx, float* y, int B, int H, int W, int C,
                       pis_stream_t stream);
int pis_maxpool2x2_bwd(const float* x, int ldx, const float* dy, const float* dskip, int ldskip,
                       float* dx, int lddx, int B, int H, int W, int C, pis_stream_t stream);

/* ---- output head: 1x1 conv C->1 + sigmoid (src/unet.py:157,206-210) ----
 * fwd: z[p] = b + sum_c x[p][c] w[c];  u[p] = 1 / (1 + exp(-z[p]))
 * bwd: d[p] = g[p] * u[p] (1 - u[p]) when u != NULL (sigmoid backward), else g[p];
 *      dx[p][c] = d[p] w[c] (x[p][c] > 0)  (ReLU backward of dec1 fused);
 *      dw[c] (+)= sum_p d[p] x[p][c];  db (+)= sum_p d[p]                         */
int pis_head_fwd(const float* x, int ldx, const float* w, const float* b, float* z, float* u,
                 int64_t npix, int C, pis_stream_t stream);
size_t pis_head_bwd_ws(int64_t npix, int C);
int pis_head_bwd(const float* x, int ldx, const float* w, const float* g, const float* u, float* dx,
                 int lddx, float* dw, float* db, int64_t npix, int C, int flags, void* ws,
                 size_t ws_bytes, pis_stream_t stream);

/* ---- fused Dice + BCE + reaction-diffusion + phase-field loss ----
 * src/loss.py:114-162, src/pde.py:49-212, src/metrics.py:38-73, src/evaluate.py:62-97.
 * p, t: (B, H, W) fp32 (C = 1). Terms are whole-batch means (src/loss.py:130-143). */
typedef struct pis_loss_params {
  float dice_w, bce_w;   /* src/loss.py:144-147                        */
  float rd_w, pf_w;      /* lambda_RD, lambda_PF; a term enters the total only if > 0 */
  float smooth;          /* Dice smoothing (1e-6)                      */
  float D, a;            /* diffusion coefficient, reaction threshold   */
  float eps;             /* phase-field interface width                */
  float thr;             /* metric threshold (0.5, strict '>')         */
  int flags;             /* PIS_LOSS_ALL_TERMS | PIS_LOSS_NO_REACTION                  */
} pis_loss_params;
#define PIS_LOSS_ALL_TERMS 1
#define PIS_LOSS_CHAIN_SIGMOID 2 /* bwd writes dL/dz = dL/dp * p (1 - p) */
#define PIS_LOSS_NO_REACTION 4   /* residual r = D Lap(u) only (src/ablation.py:53-86,107-154
                                    DiffusionOnlyLoss, use_reaction_term=False)           */
/* out_terms: [0] total [1] dice_loss [2] bce_loss [3] rd_loss [4] pf_loss [5] I=sum p t
 *            [6] P=sum p [7] T=sum t.
 * counts: [B][3] = exact (I_hat, P_hat, T) of the thresholded prediction per sample.
 * scores: [B][2] = (Dice, IoU) per sample (src/metrics.py:67-70, src/evaluate.py:91-94). */
#define PIS_LOSS_NTERMS 8
/* ws: pis_loss_ws(B, H, W) bytes of device scratch (no state between calls). */
size_t pis_loss_ws(int B, int H, int W);
int pis_loss_fwd(const float* p, const float* t, int B, int H, int W, const pis_loss_params* prm,
                 float* out_terms, int* counts, float* scores, void* ws, size_t ws_bytes,
                 pis_stream_t stream);
/* dst = grad_out * dL/dp (or dL/dz with PIS_LOSS_CHAIN_SIGMOID); grad_out is a device
 * scalar (NULL = 1).  terms = out_terms of the forward on the same p, t.          */
int pis_loss_bwd(const float* p, const float* t, int B, int H, int W, const pis_loss_params* prm,
                 const float* terms, const float* grad_out, float* dst, int flags,
                 pis_stream_t stream);

/* Loss backward fused into the head backward (src/loss.py:114-162 + src/unet.py:210 out_conv +
 * sigmoid): dz = dL/du u (1 - u) per pixel from u (B,H,W), t, terms of pis_loss_fwd, then
 * dx = dz w (x > 0), dw = sum dz x, db = sum dz as pis_head_bwd. du_out (may be NULL) receives
 * dL/du, i.e. what pis_loss_bwd writes.
 * W <= 1024. flags: PIS_ACCUMULATE (dw, db). */
/* The U-Net head (1x1 conv C -> 1 + sigmoid, src/unet.py:206-210) fused with pis_loss_fwd (replaces the
 * criterion call after model(x), src/train.py:108-110 / src/loss.py:130-160): from the head input x
 * ([B*H*W][ldx], C == 64) writes z (logits) and u = sigmoid(z) (B*H*W each, bitwise those of
 * pis_head_fwd) and every loss term / counter / score exactly as pis_loss_fwd(u, t) would; one pass
 * over x. Applicable when pis_head_loss_fwd_ok(B, H, W, C) (C == 64, W % 64 == 0, W <= 2048); else
 * use pis_head_fwd + pis_loss_fwd. Workspace pis_head_loss_fwd_ws(B, H, W) bytes. */
size_t pis_head_loss_fwd_ws(int B, int H, int W);
int pis_head_loss_fwd_ok(int B, int H, int W, int C);
int pis_head_loss_fwd(const float* x, int ldx, const float* w, const float* bias, const float* t, float* z,
                      float* u, int B, int H, int W, int C, const pis_loss_params* prm, float* out_terms,
                      int* counts, float* scores, void* ws, size_t ws_bytes, pis_stream_t stream);
size_t pis_head_loss_bwd_ws(int B, int H, int W, int C);
int pis_head_loss_bwd(const float* x, int ldx, const float* w, const float* u, const float* t,
                      float* du_out, int B, int H, int W, int C, const pis_loss_params* prm,
                      const float* terms, const float* grad_out, float* dx, int lddx, float* dw,
                      float* db, int flags, void* ws, size_t ws_bytes, pis_stream_t stream);
/* Per-pixel PDE fields of src/pde.py (any output may be NULL):
 * lap = Lap(u) (:49-79), residual = D Lap(u) + u(1-u)(u-a) (:101-122),
 * gradmag2 = gx^2 + gy^2 (:147-178), all on reflect-padded stencils.           */
int pis_pde_fields(const float* u, int B, int H, int W, float D, float a, float* lap,
                   float* residual, float* gradmag2, pis_stream_t stream);
/* Their adjoint: du = sum over the fields of (d field / du)^T g_field (any g may be NULL), so
 * PDERegularization.compute_laplacian / reaction_term / compute_residual /
 * compute_gradient_magnitude are differentiable as in the reference (src/pde.py:49-178). */
int pis_pde_fields_bwd(const float* u, const float* g_lap, const float* g_residual,
                       const float* g_gradmag2, int B, int H, int W, float D, float a, float* du,
                       pis_stream_t stream);

/* ---- decoupled AdamW over one flat parameter arena (src/train.py:658-662) ----
 * torch.optim.AdamW single-tensor semantics (torch/optim/adam.py):
 *   p *= 1 - lr*wd;  m += (1-b1)(g' - m);  v = b2 v + (1-b2) g'^2;
 *   p -= step_size * m / (sqrt(v)/bc2_sqrt + eps)     with g' = g * grad_scale.   */
int pis_adamw_step(float* p, const float* g, float* m, float* v, int64_t n, double lr, double beta1,
                   double beta2, double eps, double weight_decay, double step_size, double bc2_sqrt,
                   double grad_scale, pis_stream_t stream);

/* ---- channel sums (bias gradients): out[c] (+)= sum_p src[p*ld + c] ---- */
size_t pis_colsum_ws(int64_t npix, int C);
int pis_colsum(const float* src, int ld, int64_t npix, int C, float* out, int flags, void* ws,
               size_t ws_bytes, pis_stream_t stream);

/* ---- on-device synthetic batches (the disc generator of §8(c),
 * physics_informed_image_segmentation_amd/dataset.py:disc_sample) ----
 * discs: [B][max_discs][3] (cx, cy, r) drawn on the host from each sample's generator;
 * ndisc: [B] (device). Masks are bit-identical to the host generator's; the N(0, 0.1^2)
 * image noise is a counter-based hash of (seed, sample_ids[b] or b, pixel).
 * img, mask: (B, 1, H, W) fp32, img min-max normalised per sample. */
size_t pis_synth_ws(int B, int H, int W);
int pis_synth_discs(const float* discs, const int* ndisc, int max_discs, uint64_t seed,
                    const int64_t* sample_ids, float* img, float* mask, int B, int H, int W,
                    void* ws, size_t ws_bytes, pis_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* PIS_CAPI_H */
