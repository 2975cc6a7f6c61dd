// Lab kernels for tools/queue_probe.py (not product code): a bounded wait kernel that stands in for
// an RCCL receive posted ahead of its data -- resident, polling a device flag (vector loads only)
// until it is set or a wall-clock timeout passes -- to measure (a) whether a kernel queued on another
// HIP stream can run while it waits (streams share the process's GPU_MAX_HW_QUEUES hardware queues),
// and (b) how much a few resident polling workgroups slow a streaming kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void lab_wait_kernel(const int* flag, long long timeout_ticks) {
  const long long t0 = wall_clock64();  // 100 MHz
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) {
    if (wall_clock64() - t0 > timeout_ticks) break;
    __builtin_amdgcn_s_sleep(8);
  }
}

__global__ void lab_set_kernel(int* flag, int v) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" int lab_wait(const void* flag, double timeout_us, int n_wg, int threads, void* stream) {
  hipLaunchKernelGGL(lab_wait_kernel, dim3(n_wg), dim3(threads), 0, (hipStream_t)stream, (const int*)flag,
                     (long long)(timeout_us * 100.0));
  return (int)hipGetLastError();
}

extern "C" int lab_set(void* flag, int v, void* stream) {
  hipLaunchKernelGGL(lab_set_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, (int*)flag, v);
  return (int)hipGetLastError();
}
