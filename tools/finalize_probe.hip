// Probe: what does a one-block reduction launch cost right after a 2048-block streaming kernel?
// Variants of the consumer (run under rocprofv3 --kernel-trace to see per-kernel durations):
//   empty      : one 64-thread block, returns
//   empty1024  : one 1024-thread block, returns
//   lds1024    : 1024 threads stage 2048x9 partials in LDS (74 KB), sum (the loss finalize's shape)
//   reg256     : 256 threads, every partial loaded straight into registers, summed, no LDS staging
//   lds1024_nodbl: lds1024 with float sums instead of double
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/finalize_probe tools/finalize_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <algorithm>
#include <type_traits>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int NB = 2048;

__global__ __launch_bounds__(256) void producer(const float4* __restrict__ x, int n4, float* fpart, int* ipart) {
  float s = 0.f;
  for (int k = blockIdx.x * 256 + threadIdx.x; k < n4; k += gridDim.x * 256) {
    float4 v = x[k];
    s += v.x + v.y + v.z + v.w;
  }
  __shared__ float r[256];
  r[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x < 6) fpart[blockIdx.x * 6 + threadIdx.x] = r[threadIdx.x] + r[threadIdx.x + 64];
  else if (threadIdx.x < 9) ipart[blockIdx.x * 3 + threadIdx.x - 6] = (int)r[threadIdx.x];
}

__global__ void empty_k(float* out) { if (threadIdx.x == 1000000) out[0] = 1.f; }

template <bool DBL>
__global__ __launch_bounds__(1024) void lds1024(const float* fpart, const int* ipart, float* out) {
  __shared__ float sf[NB * 6];
  __shared__ int si[NB * 3];
  float vf[12];
  int vi[6];
#pragma unroll
  for (int j = 0; j < 12; ++j) vf[j] = fpart[threadIdx.x + 1024 * j];
#pragma unroll
  for (int j = 0; j < 6; ++j) vi[j] = ipart[threadIdx.x + 1024 * j];
#pragma unroll
  for (int j = 0; j < 12; ++j) sf[threadIdx.x + 1024 * j] = vf[j];
#pragma unroll
  for (int j = 0; j < 6; ++j) si[threadIdx.x + 1024 * j] = vi[j];
  __syncthreads();
  using T = typename std::conditional<DBL, double, float>::type;
  T s[6] = {0, 0, 0, 0, 0, 0};
  for (int k = threadIdx.x; k < NB; k += 1024)
#pragma unroll
    for (int j = 0; j < 6; ++j) s[j] += (T)sf[k * 6 + j];
  long long c = 0;
  for (int k = threadIdx.x; k < NB * 3; k += 1024) c += si[k];
#pragma unroll
  for (int j = 0; j < 6; ++j)
    for (int off = 32; off > 0; off >>= 1) s[j] += __shfl_xor(s[j], off, 64);
  __shared__ T red[16][6];
  if ((threadIdx.x & 63) == 0)
    for (int j = 0; j < 6; ++j) red[threadIdx.x >> 6][j] = s[j];
  __syncthreads();
  if (threadIdx.x == 0) {
    T t = 0;
    for (int w = 0; w < 16; ++w) t += red[w][0] + red[w][5];
    out[0] = (float)t + (float)c;
  }
}

__global__ __launch_bounds__(256) void reg256(const float* fpart, const int* ipart, float* out) {
  float vf[48];
#pragma unroll
  for (int j = 0; j < 48; ++j) vf[j] = fpart[threadIdx.x + 256 * j];
  double s = 0;
#pragma unroll
  for (int j = 0; j < 48; ++j) s += vf[j];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (float)(red[0] + red[1] + red[2] + red[3]) + ipart[0];
}

int main() {
  const size_t n = 16ull << 20;  // 16M floats = 64 MB streamed by the producer
  float *x, *fpart, *out;
  int* ipart;
  CHECK(hipMalloc(&x, n * 4));
  CHECK(hipMemset(x, 0, n * 4));
  CHECK(hipMalloc(&fpart, NB * 6 * 4));
  CHECK(hipMalloc(&ipart, NB * 3 * 4));
  CHECK(hipMalloc(&out, 64));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char* names[] = {"producer_only", "empty", "empty1024", "lds1024", "reg256", "lds1024_nodbl"};
  for (int v = 0; v < 6; ++v) {
    std::vector<float> ms;
    for (int rep = 0; rep < 30; ++rep) {
      CHECK(hipEventRecord(e0, s));
      hipLaunchKernelGGL(producer, dim3(NB), dim3(256), 0, s, (const float4*)x, (int)(n / 4), fpart, ipart);
      switch (v) {
        case 1: hipLaunchKernelGGL(empty_k, dim3(1), dim3(64), 0, s, out); break;
        case 2: hipLaunchKernelGGL(empty_k, dim3(1), dim3(1024), 0, s, out); break;
        case 3: hipLaunchKernelGGL(lds1024<true>, dim3(1), dim3(1024), 0, s, fpart, ipart, out); break;
        case 4: hipLaunchKernelGGL(reg256, dim3(1), dim3(256), 0, s, fpart, ipart, out); break;
        case 5: hipLaunchKernelGGL(lds1024<false>, dim3(1), dim3(1024), 0, s, fpart, ipart, out); break;
      }
      CHECK(hipEventRecord(e1, s));
      CHECK(hipEventSynchronize(e1));
      float t;
      CHECK(hipEventElapsedTime(&t, e0, e1));
      if (rep >= 5) ms.push_back(t * 1e3f);
    }
    std::sort(ms.begin(), ms.end());
    printf("%-14s producer+consumer median %.1f us  min %.1f us\n", names[v], ms[ms.size() / 2], ms[0]);
  }
  CHECK(hipDeviceSynchronize());
  return 0;
}
