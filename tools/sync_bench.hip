// Cross-CU synchronisation latency on the GPU this runs on (tools only, not part of the library):
//   barrier: a persistent grid (one workgroup per CU, forced by LDS) runs R rounds of a counter
//            barrier (device-scope atomic add, then bounded polls of a device-scope load);
//   relay:   workgroup i waits for flag[i - 1] to reach round r, then sets flag[i] = r (a chain
//            through every CU, consecutive block ids on different XCDs): latency per hop.
// Every wait is bounded (a lost update ends the kernel with an error count, never a hang).
// Build: hipcc -O3 --offload-arch=gfx950 tools/sync_bench.hip -o tools/wv/sync_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

constexpr int MAXPOLL = 1 << 20;

__device__ __forceinline__ int ld_dev(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

__global__ void barrier_kernel(int* cnt, int rounds, int* err) {
  extern __shared__ float pad[];
  if (threadIdx.x == 0) {
    const int G = gridDim.x;
    int bad = 0;
    for (int r = 0; r < rounds; ++r) {
      __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int n = 0;
      while (ld_dev(cnt) < (r + 1) * G && ++n < MAXPOLL) __builtin_amdgcn_s_sleep(1);
      bad += n >= MAXPOLL;
    }
    if (bad) __hip_atomic_fetch_add(err, bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pad[0] = 0.f;
  }
  __syncthreads();
}

// same, with the barrier spin done without s_sleep
__global__ void barrier_nosleep_kernel(int* cnt, int rounds, int* err) {
  extern __shared__ float pad[];
  if (threadIdx.x == 0) {
    const int G = gridDim.x;
    int bad = 0;
    for (int r = 0; r < rounds; ++r) {
      __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int n = 0;
      while (ld_dev(cnt) < (r + 1) * G && ++n < MAXPOLL) {
      }
      bad += n >= MAXPOLL;
    }
    if (bad) __hip_atomic_fetch_add(err, bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pad[0] = 0.f;
  }
  __syncthreads();
}

__global__ void relay_kernel(int* flag, int rounds, int* err) {
  extern __shared__ float pad[];
  if (threadIdx.x == 0) {
    const int i = blockIdx.x, G = gridDim.x;
    int bad = 0;
    for (int r = 1; r <= rounds; ++r) {
      // block 0 waits for the last block's previous round (a ring)
      int* src = i == 0 ? flag + G - 1 : flag + i - 1;
      const int want = i == 0 ? r - 1 : r;
      int n = 0;
      while (ld_dev(src) < want && ++n < MAXPOLL) {
      }
      bad += n >= MAXPOLL;
      __hip_atomic_store(flag + i, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (bad) __hip_atomic_fetch_add(err, bad, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    pad[0] = 0.f;
  }
  __syncthreads();
}

__global__ void empty_kernel(int* p) {
  extern __shared__ float pad[];
  if (threadIdx.x == 0 && p == nullptr) pad[0] = 0.f;
}

int main() {
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int lds = 96 * 1024;  // one workgroup per CU
  CK(hipFuncSetAttribute((const void*)barrier_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute((const void*)barrier_nosleep_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute((const void*)relay_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  CK(hipFuncSetAttribute((const void*)empty_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  int *buf = nullptr, *err = nullptr;
  CK(hipMalloc(&buf, 4096 * sizeof(int)));
  CK(hipMalloc(&err, sizeof(int)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timed = [&](auto launch, int reps) {
    float best = 1e30f;
    for (int t = 0; t < 5; ++t) {
      CK(hipMemset(buf, 0, 4096 * sizeof(int)));
      CK(hipEventRecord(a));
      launch();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    return best * 1000.f / reps;
  };
  CK(hipMemset(err, 0, sizeof(int)));
  std::printf("CUs %d\n", cus);
  for (int G : {64, 128, cus}) {
    const float e1 = timed([&] { hipLaunchKernelGGL(empty_kernel, dim3(G), dim3(256), lds, 0, buf); }, 1);
    float e10 = timed([&] {
      for (int k = 0; k < 10; ++k) hipLaunchKernelGGL(empty_kernel, dim3(G), dim3(256), lds, 0, buf);
    }, 10);
    const int R = 200;
    const float b1 = timed([&] { hipLaunchKernelGGL(barrier_kernel, dim3(G), dim3(256), lds, 0, buf, R, err); }, R);
    const float b2 = timed([&] { hipLaunchKernelGGL(barrier_nosleep_kernel, dim3(G), dim3(256), lds, 0, buf, R, err); }, R);
    const int RR = 20;
    const float rl = timed([&] { hipLaunchKernelGGL(relay_kernel, dim3(G), dim3(256), lds, 0, buf, RR, err); }, RR * G);
    std::printf("grid %4d: empty launch %.2f us (alone) %.2f us (10 back to back); barrier %.2f us (s_sleep) %.2f us (spin); relay hop %.3f us\n",
                G, e1, e10, b1, b2, rl);
  }
  int herr = 0;
  CK(hipMemcpy(&herr, err, sizeof(int), hipMemcpyDeviceToHost));
  std::printf("expired waits: %d\n", herr);
  return herr ? 2 : 0;
}
