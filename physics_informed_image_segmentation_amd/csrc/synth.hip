// On-device synthetic cell-image batches: the disc generator of
// SURVEY §8(c) / dataset.py:disc_sample rasterised on the GPU, so a data-parallel run does
// not wait on host workers (the host generator spends ~20 ms per 512^2 sample in Python).
//
//   mask(y, x) = OR_k [ (x - cx_k)^2 + (y - cy_k)^2 <= r_k^2 ]
//   raw        = 0.2 + 0.6 mask + 0.1 n,  n ~ N(0, 1)
//   img        = (raw - min raw) / (max raw - min raw + 1e-8)   per sample
//
// The disc parameters (cx, cy, r per sample) are drawn on the host from the sample's own
// torch.Generator in the host generator's order, and the disc test is evaluated with
// correctly rounded, uncontracted fp32 ops in torch's order ((dx*dx) + (dy*dy) <= r*r), so
// the MASKS are bit-identical to the host generator's. The noise is a counter-based hash
// (splitmix64 -> Box-Muller) of (seed, sample, pixel): deterministic and shard-independent,
// but not torch.randn's stream.
#include "common.h"

namespace pis {

constexpr int SYN_PIX = 1024;  // pixels per block (256 threads x 4)

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float gauss(uint64_t key) {
  const uint64_t h = splitmix64(key);
  const float u1 = ((uint32_t)(h >> 40) + 1u) * (1.0f / 16777217.0f);  // (0, 1]
  const float u2 = (uint32_t)(h & 0xFFFFFFu) * (1.0f / 16777216.0f);   // [0, 1)
  return sqrtf(-2.f * logf(u1)) * cosf(6.2831853071795864f * u2);
}

struct SynthArgs {
  const float* discs;  // [B][maxd][3] (cx, cy, r)
  const int* ndisc;    // [B]
  int maxd;
  uint64_t seed;
  const int64_t* sample_ids;  // [B] global sample index (the noise key), or NULL = b
  float* img;
  float* mask;
  int B, H, W, nblk;
  float* part;  // [B][nblk][2] (min, max)
};

__global__ __launch_bounds__(256) void synth_raw_kernel(SynthArgs a) {
  __shared__ float sd[64 * 3];
  __shared__ float red[2][4];
  const int b = blockIdx.y, nd = min(a.ndisc[b], 64);
  for (int i = threadIdx.x; i < nd * 3; i += 256) sd[i] = a.discs[((size_t)b * a.maxd) * 3 + i];
  __syncthreads();
  const int64_t npx = (int64_t)a.H * a.W;
  const uint64_t sid = a.sample_ids ? (uint64_t)a.sample_ids[b] : (uint64_t)b;
  float mn = INFINITY, mx = -INFINITY;
  const int64_t p0 = (int64_t)blockIdx.x * SYN_PIX + threadIdx.x * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t p = p0 + j;
    if (p >= npx) break;
    const int y = (int)(p / a.W), x = (int)(p - (int64_t)y * a.W);
    bool in = false;
    for (int k = 0; k < nd; ++k) {
      const float dx = __fsub_rn((float)x, sd[3 * k]), dy = __fsub_rn((float)y, sd[3 * k + 1]);
      const float r = sd[3 * k + 2];
      in |= __fadd_rn(__fmul_rn(dx, dx), __fmul_rn(dy, dy)) <= __fmul_rn(r, r);
    }
    const float m = in ? 1.f : 0.f;
    const float n = gauss((a.seed * 0x2545F4914F6CDD1Dull) ^ (sid << 32) ^ (uint64_t)p);
    const float raw = __fadd_rn(__fadd_rn(0.2f, __fmul_rn(0.6f, m)), __fmul_rn(0.1f, n));
    a.mask[(size_t)b * npx + p] = m;
    a.img[(size_t)b * npx + p] = raw;
    mn = fminf(mn, raw);
    mx = fmaxf(mx, raw);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, off, 64));
    mx = fmaxf(mx, __shfl_xor(mx, off, 64));
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wv] = mn;
    red[1][wv] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float* o = a.part + ((size_t)b * a.nblk + blockIdx.x) * 2;
    o[0] = fminf(fminf(red[0][0], red[0][1]), fminf(red[0][2], red[0][3]));
    o[1] = fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3]));
  }
}

__global__ __launch_bounds__(256) void synth_norm_kernel(SynthArgs a) {
  __shared__ float red[2][4];
  const int b = blockIdx.y;
  float mn = INFINITY, mx = -INFINITY;
  for (int i = threadIdx.x; i < a.nblk; i += 256) {
    mn = fminf(mn, a.part[((size_t)b * a.nblk + i) * 2]);
    mx = fmaxf(mx, a.part[((size_t)b * a.nblk + i) * 2 + 1]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mn = fminf(mn, __shfl_xor(mn, off, 64));
    mx = fmaxf(mx, __shfl_xor(mx, off, 64));
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wv] = mn;
    red[1][wv] = mx;
  }
  __syncthreads();
  mn = fminf(fminf(red[0][0], red[0][1]), fminf(red[0][2], red[0][3]));
  mx = fmaxf(fmaxf(red[1][0], red[1][1]), fmaxf(red[1][2], red[1][3]));
  const float den = __fadd_rn(__fsub_rn(mx, mn), 1e-8f);
  const int64_t npx = (int64_t)a.H * a.W;
  const int64_t p0 = (int64_t)blockIdx.x * SYN_PIX + threadIdx.x * 4;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t p = p0 + j;
    if (p >= npx) break;
    float* q = a.img + (size_t)b * npx + p;
    *q = __fdiv_rn(__fsub_rn(*q, mn), den);
  }
}

}  // namespace pis

using namespace pis;

extern "C" size_t pis_synth_ws(int B, int H, int W) {
  return (size_t)B * cdiv((int64_t)H * W, SYN_PIX) * 2 * sizeof(float) + 256;
}

extern "C" int pis_synth_discs(const float* discs, const int* ndisc, int max_discs, uint64_t seed,
                               const int64_t* sample_ids, float* img, float* mask, int B, int H, int W,
                               void* ws, size_t ws_bytes, pis_stream_t stream) {
  PIS_CHECK_ARG(discs && ndisc && img && mask && B > 0 && H > 0 && W > 0 && max_discs > 0 && max_discs <= 64,
                "pis_synth_discs: bad arguments (1 <= max_discs <= 64)");
  PIS_CHECK_ARG(ws && ws_bytes >= pis_synth_ws(B, H, W), "pis_synth_discs: workspace too small");
  PIS_CHECK_ARG(B <= 65535, "pis_synth_discs: B > 65535");
  SynthArgs a{};
  a.discs = discs; a.ndisc = ndisc; a.maxd = max_discs; a.seed = seed; a.sample_ids = sample_ids;
  a.img = img; a.mask = mask; a.B = B; a.H = H; a.W = W;
  a.nblk = (int)cdiv((int64_t)H * W, SYN_PIX);
  a.part = (float*)ws;
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid(a.nblk, B);
  hipLaunchKernelGGL(synth_raw_kernel, grid, dim3(256), 0, s, a);
  int rc = launch_status("synth_raw");
  if (rc) return rc;
  hipLaunchKernelGGL(synth_norm_kernel, grid, dim3(256), 0, s, a);
  return launch_status("synth_norm");
}
