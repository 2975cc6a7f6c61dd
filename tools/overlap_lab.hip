// Overlap lab: do two kernels in parallel hipGraph branches (or on two streams) run
// concurrently on this ROCm, and in which order do their workgroups start?
//   A (producer): every workgroup spins ~`us` microseconds (s_memrealtime), then one lane adds
//                 to a counter (agent scope).
//   B (consumer): every workgroup polls the counter (sc1 loads, s_sleep, bounded) until it
//                 reaches A's grid size; records the polls it needed (or a give-up).
// Printed per mode: B's give-ups (0 = B saw A finish, i.e. both ran concurrently or A first),
// total wall time.  hipcc --offload-arch=gfx950 -O3 tools/overlap_lab.hip -o /tmp/overlap_lab
#include <hip/hip_runtime.h>

#include <stdio.h>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      printf("%s failed: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      return 1;                                                                 \
    }                                                                           \
  } while (0)

__global__ void producer(unsigned* cnt, int us) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)us * 100) __builtin_amdgcn_s_sleep(2);
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void consumer(const unsigned* cnt, unsigned target, int* gaveup, unsigned* polls_max) {
  if (threadIdx.x == 0) {
    unsigned n = 0;
    while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(8);
      if (++n > 2000000u) {
        atomicAdd(gaveup, 1);
        break;
      }
    }
    atomicMax(polls_max, n);
  }
}

__global__ void reset(unsigned* cnt, int* gaveup, unsigned* polls) {
  *cnt = 0;
  *gaveup = 0;
  *polls = 0;
}

int main() {
  unsigned *cnt, *polls;
  int* gaveup;
  CK(hipMalloc(&cnt, 256));
  CK(hipMalloc(&gaveup, 256));
  CK(hipMalloc(&polls, 256));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t fork, join, t0, t1;
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  const int NA = 512, NB = 256, US = 200;
  for (int mode = 0; mode < 4; ++mode) {
    // mode 0: graph, A captured first; 1: graph, B captured first; 2: eager A then B;
    // 3: eager B then A
    hipLaunchKernelGGL(reset, dim3(1), dim3(1), 0, s1, cnt, gaveup, polls);
    CK(hipStreamSynchronize(s1));
    hipGraphExec_t ge = nullptr;
    auto enqueue = [&](bool b_first) {
      CK(hipEventRecord(fork, s1));
      CK(hipStreamWaitEvent(s2, fork, 0));
      if (b_first) {
        hipLaunchKernelGGL(consumer, dim3(NB), dim3(256), 0, s2, cnt, (unsigned)NA, gaveup, polls);
        hipLaunchKernelGGL(producer, dim3(NA), dim3(256), 0, s1, cnt, US);
      } else {
        hipLaunchKernelGGL(producer, dim3(NA), dim3(256), 0, s1, cnt, US);
        hipLaunchKernelGGL(consumer, dim3(NB), dim3(256), 0, s2, cnt, (unsigned)NA, gaveup, polls);
      }
      CK(hipEventRecord(join, s2));
      CK(hipStreamWaitEvent(s1, join, 0));
      return 0;
    };
    if (mode < 2) {
      hipGraph_t g;
      CK(hipStreamBeginCapture(s1, hipStreamCaptureModeGlobal));
      if (enqueue(mode == 1)) return 1;
      CK(hipStreamEndCapture(s1, &g));
      CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CK(hipEventRecord(t0, s1));
      CK(hipGraphLaunch(ge, s1));
      CK(hipEventRecord(t1, s1));
    } else {
      CK(hipEventRecord(t0, s1));
      if (enqueue(mode == 3)) return 1;
      CK(hipEventRecord(t1, s1));
    }
    CK(hipStreamSynchronize(s1));
    CK(hipDeviceSynchronize());
    int h_gu = -1;
    unsigned h_p = 0, h_c = 0;
    float ms = 0.f;
    CK(hipMemcpy(&h_gu, gaveup, 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&h_p, polls, 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&h_c, cnt, 4, hipMemcpyDeviceToHost));
    CK(hipEventElapsedTime(&ms, t0, t1));
    printf("mode %d (%s, %s first): consumer give-ups %d / %d, max polls %u, producer count %u, %.3f ms\n", mode,
           mode < 2 ? "graph" : "eager", (mode & 1) ? "B" : "A", h_gu, NB, h_p, h_c, ms);
  }
  return 0;
}
