// Persistent-chain economics lab (read-only, no MFMA): does one launch that streams the o, gate/up
// and down weight bytes of a Qwen3-8B decode layer (33.9 / 201.9 / 101.3 MB) as three phases
// separated by in-launch hand-offs beat three launches of the same streams?  The phases read each
// workgroup's contiguous slice with a register ring of 16-B loads (the decode GEMVs' weight
// stream); before each hand-off wait a phase's successor already has its first ring stages in
// flight (the persistent design's prefetch credit).  Hand-off = per-XCD sharded arrival counter
// (agent atomic add by one lane after the workgroup's loads retire), polled by one lane with sc1
// loads and s_sleep, bounded (a wait that gives up sets a flag and the run is reported invalid).
// Sets of buffers are rotated so no launch finds its bytes in the 256 MB Infinity Cache.
//   hipcc --offload-arch=gfx950 -O3 -std=c++20 tools/chain_lab.hip -o tools/labbin/chain_lab
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int NPH = 3;
struct Chain {
  const u32x4* w[NPH];
  long long slice[NPH];  // bytes per workgroup (a multiple of 1 KiB * waves)
};

// one phase of one workgroup: NW waves stream the workgroup's slice in 1 KiB tiles (wave w: tiles
// w, w + NW, ...), D tiles in flight per wave.  PRE: the first D tiles were issued by the caller.
template <int NW, int D>
__device__ __forceinline__ unsigned stream_slice(const u32x4* base, long long bytes, int wave, int lane,
                                                 u32x4 (&r)[D], bool pre) {
  // straight-line passes of D unconditional loads (addresses past the wave's last tile re-read
  // it): hipcc then counts every wait (vmcnt(D - 1)) instead of draining the ring
  const long long ntiles = bytes / 1024;
  const long long nper = (ntiles - wave + NW - 1) / NW;
  auto addr = [&](long long j) { return base + (wave + (j < nper ? j : nper - 1) * NW) * 64 + lane; };
  unsigned x = 0;
  if (!pre) {
#pragma unroll
    for (int d = 0; d < D; ++d) r[d] = __builtin_nontemporal_load(addr(d));
  }
  for (long long j = 0; j < nper; j += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      x ^= r[d][0] ^ r[d][1] ^ r[d][2] ^ r[d][3];
      r[d] = __builtin_nontemporal_load(addr(j + d + D));
    }
  }
  return x;
}

template <int NW, int D>
__global__ __launch_bounds__(NW * 64) void phase_kernel(const u32x4* w, long long slice, unsigned* sink) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  u32x4 r[D];
  const unsigned x = stream_slice<NW, D>(w + (long long)blockIdx.x * slice / 16, slice, wave, lane, r, false);
  if (x == 0x9e3779b9u) sink[0] = x;
}

// the same stream plus, per weight tile, one 1 KiB activation-fragment load from a small
// L2-resident buffer (the decode GEMV's A operand: every workgroup reads all of it)
template <int NW, int D, int ROTA = 0, int VAR = 0>
__global__ __launch_bounds__(NW * 64) void phase_a_kernel(const u32x4* w, long long slice, const u32x4* a,
                                                          long long a_tiles, unsigned* sink) {
  // ROTA: workgroup n starts its activation walk at tile (n * ROTA) % a_tiles, so concurrent CUs
  // read different lines (every workgroup walking A in the same order hits the same L2 channel)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u32x4* base = w + (long long)blockIdx.x * slice / 16;
  const long long ntiles = slice / 1024;
  const long long nper = (ntiles - wave + NW - 1) / NW;
  auto addr = [&](long long j) { return base + (wave + (j < nper ? j : nper - 1) * NW) * 64 + lane; };
  const long long rot = ((long long)blockIdx.x * ROTA) % a_tiles;
  auto aaddr = [&](long long j) { return a + ((wave + (j < nper ? j : nper - 1) * NW + rot) % a_tiles) * 64 + lane; };
  // VAR 0: A then W per stage; 1: W then A; 2: A from LDS (the workgroup copies A in first;
  // a_tiles <= 128)
  u32x4 r[D], ra[D];
  unsigned x = 0;
  __shared__ u32x4 als[VAR == 2 ? 128 * 64 : 1];
  if constexpr (VAR == 2) {
    for (int i = threadIdx.x; i < a_tiles * 64; i += NW * 64) als[i] = a[i];
    __syncthreads();
  }
  auto lda = [&](long long j) {
    if constexpr (VAR == 2)
      return als[((wave + (j < nper ? j : nper - 1) * NW + rot) % a_tiles) * 64 + lane];
    else
      return aaddr(j)[0];
  };
#pragma unroll
  for (int d = 0; d < D; ++d) {
    if (VAR != 1) ra[d] = lda(d);
    r[d] = __builtin_nontemporal_load(addr(d));
    if (VAR == 1) ra[d] = lda(d);
  }
  for (long long j = 0; j < nper; j += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      x ^= r[d][0] ^ r[d][1] ^ r[d][2] ^ r[d][3] ^ ra[d][0] ^ ra[d][3];
      if (VAR != 1) ra[d] = lda(j + d + D);
      r[d] = __builtin_nontemporal_load(addr(j + d + D));
      if (VAR == 1) ra[d] = lda(j + d + D);
    }
  }
  if (x == 0x9e3779b9u) sink[0] = x;
}

// cache-policy variants of the A + W stream (buffer loads, aux bits: 1 sc0, 2 nt, 16 sc1)
template <int NW, int D, int AW, int AA>
__global__ __launch_bounds__(NW * 64) void phase_pol_kernel(const u32x4* w, long long slice, const u32x4* a,
                                                            long long a_tiles, unsigned* sink) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long ntiles = slice / 1024;
  const long long nper = (ntiles - wave + NW - 1) / NW;
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)(w + (long long)blockIdx.x * slice / 16), 0, (int)slice, 0x00020000);
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc((void*)a, 0, (int)(a_tiles * 1024), 0x00020000);
  auto wo = [&](long long j) { return (int)((wave + (j < nper ? j : nper - 1) * NW) * 1024 + lane * 16); };
  auto ao = [&](long long j) { return (int)(((wave + (j < nper ? j : nper - 1) * NW) % a_tiles) * 1024 + lane * 16); };
  u32x4 r[D], ra[D];
  unsigned x = 0;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    ra[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ar, ao(d), 0, AA));
    r[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, wo(d), 0, AW));
  }
  for (long long j = 0; j < nper; j += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      x ^= r[d][0] ^ r[d][1] ^ r[d][2] ^ r[d][3] ^ ra[d][0] ^ ra[d][3];
      ra[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ar, ao(j + d + D), 0, AA));
      r[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, wo(j + d + D), 0, AW));
    }
  }
  if (x == 0x9e3779b9u) sink[0] = x;
}

// A staged into LDS by LDS-DMA (the whole 128 KiB, 16 pieces per wave) right behind the weight
// ring's prologue, then read with ds_read_b128: no vector-memory instruction for A in the loop
template <int NW, int D>
__global__ __launch_bounds__(NW * 64) void phase_alds_kernel(const u32x4* w, long long slice, const u32x4* a,
                                                             long long a_tiles, unsigned* sink) {
  extern __shared__ __attribute__((aligned(16))) u32x4 alds[];
  typedef __attribute__((address_space(3))) void* lds_ptr;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long ntiles = slice / 1024;
  const long long nper = (ntiles - wave + NW - 1) / NW;
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)(w + (long long)blockIdx.x * slice / 16), 0, (int)slice, 0x00020000);
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc((void*)a, 0, (int)(a_tiles * 1024), 0x00020000);
  auto wo = [&](long long j) { return (int)((wave + (j < nper ? j : nper - 1) * NW) * 1024 + lane * 16); };
  auto ai = [&](long long j) { return (int)(((wave + (j < nper ? j : nper - 1) * NW) % a_tiles) * 64 + lane); };
  u32x4 r[D];
  unsigned x = 0;
#pragma unroll
  for (int d = 0; d < D; ++d) r[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, wo(d), 0, 2));
  for (int t = wave; t < a_tiles; t += NW)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ar, (lds_ptr)(alds + t * 64), 16, lane * 16, t * 1024, 0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (long long j = 0; j < nper; j += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const u32x4 av = alds[ai(j + d)];
      x ^= r[d][0] ^ r[d][1] ^ r[d][2] ^ r[d][3] ^ av[0] ^ av[3];
      r[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, wo(j + d + D), 0, 2));
    }
  }
  if (x == 0x9e3779b9u) sink[0] = x;
}

// A held in registers: each wave loads all NT of its activation tiles right behind the weight
// ring's prologue, then the loop streams weights only (o-shaped: 16 tiles per wave)
template <int NW, int D, int NT>
__global__ __launch_bounds__(NW * 64) void phase_areg_kernel(const u32x4* w, long long slice, const u32x4* a,
                                                             long long a_tiles, unsigned* sink) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t wr =
      __builtin_amdgcn_make_buffer_rsrc((void*)(w + (long long)blockIdx.x * slice / 16), 0, (int)slice, 0x00020000);
  const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc((void*)a, 0, (int)(a_tiles * 1024), 0x00020000);
  auto wo = [&](int j) { return (wave + (j < NT ? j : NT - 1) * NW) * 1024 + lane * 16; };
  u32x4 r[D], ra[NT];
  unsigned x = 0;
#pragma unroll
  for (int d = 0; d < D; ++d) r[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, wo(d), 0, 2));
#pragma unroll
  for (int j = 0; j < NT; ++j)
    ra[j] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(ar, ((wave + j * NW) % (int)a_tiles) * 1024 + lane * 16, 0, 0));
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int d = j % D;
    x ^= r[d][0] ^ r[d][1] ^ r[d][2] ^ r[d][3] ^ ra[j][0] ^ ra[j][3];
    r[d] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, wo(j + D), 0, 2));
  }
  if (x == 0x9e3779b9u) sink[0] = x;
}

__device__ __forceinline__ int xcc_id() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 3)" : "=s"(v));
  return v;
}

// counters: [NPH - 1 edges][8 shards] u32, monotonic over launches (target = (it + 1) * gridDim.x)
template <int NW, int D, int WAIT, int P>
__device__ __forceinline__ void chain_edge(const u32x4* nxt, long long nslice, unsigned* counters, unsigned target,
                                           int shard, int wave, int lane, u32x4 (&r)[D], unsigned* flag) {
  __shared__ int go;
  // arrive: this workgroup's phase-P work is done (every wave's loads retired)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(counters + P * 8 + shard, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // prefetch credit: the next phase's first D tiles of every wave go out before the wait
  const u32x4* nb = nxt + (long long)blockIdx.x * nslice / 16;
  const long long nt = nslice / 1024;
  const long long nper = (nt - wave + NW - 1) / NW;
#pragma unroll
  for (int d = 0; d < D; ++d) r[d] = __builtin_nontemporal_load(nb + (wave + (d < nper ? d : nper - 1) * NW) * 64 + lane);
  if (WAIT && threadIdx.x == 0) {
    long spins = 0;
    for (;;) {
      unsigned s = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) s += __hip_atomic_load(counters + P * 8 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (s >= target || __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
      if (++spins > (1l << 18)) {
        atomicOr(flag, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    go = 1;
  }
  __syncthreads();
}

template <int NW, int D, int WAIT = 1>
__global__ __launch_bounds__(NW * 64, 1) void chain_kernel(const u32x4* w0, const u32x4* w1, const u32x4* w2,
                                                           long long s0, long long s1, long long s2,
                                                           unsigned* counters, int it, unsigned* sink,
                                                           unsigned* flag) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  u32x4 r[D];
  const int shard = xcc_id();
  const unsigned target = (unsigned)(it + 1) * gridDim.x;
  unsigned x = stream_slice<NW, D>(w0 + (long long)blockIdx.x * s0 / 16, s0, wave, lane, r, false);
  chain_edge<NW, D, WAIT, 0>(w1, s1, counters, target, shard, wave, lane, r, flag);
  x ^= stream_slice<NW, D>(w1 + (long long)blockIdx.x * s1 / 16, s1, wave, lane, r, true);
  chain_edge<NW, D, WAIT, 1>(w2, s2, counters, target, shard, wave, lane, r, flag);
  x ^= stream_slice<NW, D>(w2 + (long long)blockIdx.x * s2 / 16, s2, wave, lane, r, true);
  if (x == 0x9e3779b9u) sink[0] = x;
}

int main() {
  const long long bytes[NPH] = {33947648ll, 201850880ll, 101318656ll};  // o, gate/up, down (+ tails)
  const int ROT = 3;
  std::vector<u32x4*> sets[NPH];
  for (int p = 0; p < NPH; ++p)
    for (int s = 0; s < ROT; ++s) {
      u32x4* b;
      CHECK(hipMalloc(&b, bytes[p] + (1 << 20)));
      CHECK(hipMemset(b, 0x11 * (s + 1), bytes[p] + (1 << 20)));
      sets[p].push_back(b);
    }
  unsigned *sink, *counters, *flag;
  CHECK(hipMalloc(&sink, 64));
  CHECK(hipMalloc(&counters, 4096));
  CHECK(hipMalloc(&flag, 4));
  CHECK(hipMemset(counters, 0, 4096));
  CHECK(hipMemset(flag, 0, 4));
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  printf("CUs %d\n", ncu);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto fn) {
    for (int i = 0; i < 2 * ROT; ++i) fn(i);
    CHECK(hipDeviceSynchronize());
    const int n = 30 * ROT;
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < n; ++i) fn(2 * ROT + i);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    unsigned f = 0;
    CHECK(hipMemcpy(&f, flag, 4, hipMemcpyDeviceToHost));
    printf("  %-44s %8.2f us per chain%s\n", name, ms * 1e3f / n, f ? "  (A WAIT GAVE UP: invalid)" : "");
  };
  // the engine's launch geometries: o 256 x 8 waves, gate/up 768 x 4, down 256 x 8
  timeit("3 launches, engine geometry (D 3)", [&](int i) {
    const int s = i % ROT;
    hipLaunchKernelGGL((phase_kernel<8, 3>), dim3(256), dim3(512), 0, 0, sets[0][s], bytes[0] / 256, sink);
    hipLaunchKernelGGL((phase_kernel<4, 3>), dim3(768), dim3(256), 0, 0, sets[1][s], bytes[1] / 768, sink);
    hipLaunchKernelGGL((phase_kernel<8, 3>), dim3(256), dim3(512), 0, 0, sets[2][s], bytes[2] / 256, sink);
  });
  timeit("o alone (256 x 8)", [&](int i) {
    hipLaunchKernelGGL((phase_kernel<8, 3>), dim3(256), dim3(512), 0, 0, sets[0][i % ROT], bytes[0] / 256, sink);
  });
  timeit("gate/up alone (768 x 4)", [&](int i) {
    hipLaunchKernelGGL((phase_kernel<4, 3>), dim3(768), dim3(256), 0, 0, sets[1][i % ROT], bytes[1] / 768, sink);
  });
  timeit("down alone (256 x 8)", [&](int i) {
    hipLaunchKernelGGL((phase_kernel<8, 3>), dim3(256), dim3(512), 0, 0, sets[2][i % ROT], bytes[2] / 256, sink);
  });
  u32x4* abuf;
  CHECK(hipMalloc(&abuf, 393216));
  CHECK(hipMemset(abuf, 0x22, 393216));
  timeit("o-like + A loads (128 KiB A)", [&](int i) {
    hipLaunchKernelGGL((phase_a_kernel<8, 3>), dim3(256), dim3(512), 0, 0, sets[0][i % ROT], bytes[0] / 256, abuf, 128ll,
                       sink);
  });
  timeit("down-like + A loads (384 KiB A)", [&](int i) {
    hipLaunchKernelGGL((phase_a_kernel<8, 3>), dim3(256), dim3(512), 0, 0, sets[2][i % ROT], bytes[2] / 256, abuf, 384ll,
                       sink);
  });
  timeit("gate/up-like + A loads (128 KiB A)", [&](int i) {
    hipLaunchKernelGGL((phase_a_kernel<4, 3>), dim3(768), dim3(256), 0, 0, sets[1][i % ROT], bytes[1] / 768, abuf, 128ll,
                       sink);
  });
  timeit("o-like + A loads, D 4", [&](int i) {
    hipLaunchKernelGGL((phase_a_kernel<8, 4>), dim3(256), dim3(512), 0, 0, sets[0][i % ROT], bytes[0] / 256, abuf, 128ll,
                       sink);
  });
  timeit("down-like + A loads, D 4", [&](int i) {
    hipLaunchKernelGGL((phase_a_kernel<8, 4>), dim3(256), dim3(512), 0, 0, sets[2][i % ROT], bytes[2] / 256, abuf, 384ll,
                       sink);
  });
  auto pol = [&](const char* name, auto kern, int ph, long long at) {
    timeit(name, [&](int i) {
      hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, sets[ph][i % ROT], bytes[ph] / 256, abuf, at, sink);
    });
  };
  CHECK(hipFuncSetAttribute((const void*)phase_alds_kernel<8, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CHECK(hipFuncSetAttribute((const void*)phase_alds_kernel<8, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  timeit("o-like, A by LDS-DMA + ds_read (D 3)", [&](int i) {
    hipLaunchKernelGGL((phase_alds_kernel<8, 3>), dim3(256), dim3(512), 131072, 0, sets[0][i % ROT], bytes[0] / 256, abuf,
                       128ll, sink);
  });
  timeit("o-like, A by LDS-DMA + ds_read (D 4)", [&](int i) {
    hipLaunchKernelGGL((phase_alds_kernel<8, 4>), dim3(256), dim3(512), 131072, 0, sets[0][i % ROT], bytes[0] / 256, abuf,
                       128ll, sink);
  });
  timeit("o-like, A in registers up front (D 3)", [&](int i) {
    hipLaunchKernelGGL((phase_areg_kernel<8, 3, 16>), dim3(256), dim3(512), 0, 0, sets[0][i % ROT], bytes[0] / 256 / 1024 * 1024,
                       abuf, 128ll, sink);
  });
  timeit("o-like, A in registers up front (D 4)", [&](int i) {
    hipLaunchKernelGGL((phase_areg_kernel<8, 4, 16>), dim3(256), dim3(512), 0, 0, sets[0][i % ROT], bytes[0] / 256 / 1024 * 1024,
                       abuf, 128ll, sink);
  });
  timeit("o alone D 4", [&](int i) {
    hipLaunchKernelGGL((phase_kernel<8, 4>), dim3(256), dim3(512), 0, 0, sets[0][i % ROT], bytes[0] / 256, sink);
  });
  pol("o-like pol W nt, A plain, A = 1 KiB (L1 hits)", phase_pol_kernel<8, 3, 2, 0>, 0, 1ll);
  pol("down-like pol W nt, A plain, A = 1 KiB (L1 hits)", phase_pol_kernel<8, 3, 2, 0>, 2, 1ll);
  pol("o-like pol W nt, A plain, A = 16 KiB", phase_pol_kernel<8, 3, 2, 0>, 0, 16ll);
  pol("o-like pol W nt, A plain", phase_pol_kernel<8, 3, 2, 0>, 0, 128ll);
  pol("o-like pol W nt, A nt", phase_pol_kernel<8, 3, 2, 2>, 0, 128ll);
  pol("o-like pol W nt, A sc1", phase_pol_kernel<8, 3, 2, 16>, 0, 128ll);
  pol("o-like pol W plain, A plain", phase_pol_kernel<8, 3, 0, 0>, 0, 128ll);
  pol("o-like pol W sc1, A plain", phase_pol_kernel<8, 3, 16, 0>, 0, 128ll);
  pol("o-like pol W nt, A plain, D 5", phase_pol_kernel<8, 5, 2, 0>, 0, 128ll);
  pol("down-like pol W nt, A plain", phase_pol_kernel<8, 3, 2, 0>, 2, 384ll);
  pol("down-like pol W nt, A nt", phase_pol_kernel<8, 3, 2, 2>, 2, 384ll);
  pol("down-like pol W nt, A sc1", phase_pol_kernel<8, 3, 2, 16>, 2, 384ll);
  pol("down-like pol W plain, A plain", phase_pol_kernel<8, 3, 0, 0>, 2, 384ll);
  pol("down-like pol W nt, A plain, D 5", phase_pol_kernel<8, 5, 2, 0>, 2, 384ll);
  timeit("o-like + A, W first", [&](int i) {
    hipLaunchKernelGGL((phase_a_kernel<8, 3, 0, 1>), dim3(256), dim3(512), 0, 0, sets[0][i % ROT], bytes[0] / 256, abuf,
                       128ll, sink);
  });
  timeit("down-like + A, W first", [&](int i) {
    hipLaunchKernelGGL((phase_a_kernel<8, 3, 0, 1>), dim3(256), dim3(512), 0, 0, sets[2][i % ROT], bytes[2] / 256, abuf,
                       384ll, sink);
  });
  timeit("o-like + A from LDS", [&](int i) {
    hipLaunchKernelGGL((phase_a_kernel<8, 3, 0, 2>), dim3(256), dim3(512), 0, 0, sets[0][i % ROT], bytes[0] / 256, abuf,
                       128ll, sink);
  });
  for (int rk : {1, 3, 13, 37}) {
    char nm[80];
    auto run_rot = [&](auto kern, const char* what, int nw, int grid, int ph, long long at) {
      snprintf(nm, sizeof nm, "%s + A, rotated x%d", what, rk);
      timeit(nm, [&](int i) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(nw * 64), 0, 0, sets[ph][i % ROT], bytes[ph] / grid, abuf, at, sink);
      });
    };
    if (rk == 1) {
      run_rot(phase_a_kernel<8, 3, 1>, "o-like", 8, 256, 0, 128ll);
      run_rot(phase_a_kernel<8, 3, 1>, "down-like", 8, 256, 2, 384ll);
    } else if (rk == 3) {
      run_rot(phase_a_kernel<8, 3, 3>, "o-like", 8, 256, 0, 128ll);
      run_rot(phase_a_kernel<8, 3, 3>, "down-like", 8, 256, 2, 384ll);
    } else if (rk == 13) {
      run_rot(phase_a_kernel<8, 3, 13>, "o-like", 8, 256, 0, 128ll);
      run_rot(phase_a_kernel<8, 3, 13>, "down-like", 8, 256, 2, 384ll);
      run_rot(phase_a_kernel<4, 3, 13>, "gate/up-like", 4, 768, 1, 128ll);
    } else {
      run_rot(phase_a_kernel<8, 3, 37>, "o-like", 8, 256, 0, 128ll);
      run_rot(phase_a_kernel<8, 3, 37>, "down-like", 8, 256, 2, 384ll);
      run_rot(phase_a_kernel<4, 3, 37>, "gate/up-like", 4, 768, 1, 128ll);
    }
  }
  // one grid of ncu workgroups for every phase (the persistent geometry), as 3 launches
  const long long sl[NPH] = {bytes[0] / ncu / 12288 * 12288, bytes[1] / ncu / 12288 * 12288,
                             bytes[2] / ncu / 12288 * 12288};
  timeit("3 launches, ncu x 12 waves (D 3)", [&](int i) {
    const int s = i % ROT;
    for (int p = 0; p < NPH; ++p)
      hipLaunchKernelGGL((phase_kernel<12, 3>), dim3(ncu), dim3(768), 0, 0, sets[p][s], sl[p], sink);
  });
  int it = 0;
  auto chain = [&](const char* name, auto kern, int threads) {
    timeit(name, [&](int i) {
      const int s = i % ROT;
      // 96 KiB of (unused) LDS: one workgroup per CU, every workgroup resident
      hipLaunchKernelGGL(kern, dim3(ncu), dim3(threads), 98304, 0, sets[0][s], sets[1][s], sets[2][s], sl[0], sl[1],
                         sl[2], counters, it++, sink, flag);
    });
  };
  CHECK(hipFuncSetAttribute((const void*)chain_kernel<12, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, 98304));
  CHECK(hipFuncSetAttribute((const void*)chain_kernel<12, 5>, hipFuncAttributeMaxDynamicSharedMemorySize, 98304));
  CHECK(hipFuncSetAttribute((const void*)chain_kernel<8, 4>, hipFuncAttributeMaxDynamicSharedMemorySize, 98304));
  CHECK(hipFuncSetAttribute((const void*)chain_kernel<16, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, 98304));
  chain("persistent chain, ncu x 12 waves (D 3)", chain_kernel<12, 3>, 768);
  CHECK(hipMemset(counters, 0, 4096));
  it = 0;
  chain("persistent chain, ncu x 12 waves (D 5)", chain_kernel<12, 5>, 768);
  CHECK(hipMemset(counters, 0, 4096));
  it = 0;
  chain("persistent chain, ncu x 8 waves (D 4)", chain_kernel<8, 4>, 512);
  CHECK(hipMemset(counters, 0, 4096));
  it = 0;
  chain("persistent chain, ncu x 16 waves (D 3)", chain_kernel<16, 3>, 1024);
  CHECK(hipFuncSetAttribute((const void*)chain_kernel<12, 3, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 98304));
  CHECK(hipFuncSetAttribute((const void*)chain_kernel<12, 5, 0>, hipFuncAttributeMaxDynamicSharedMemorySize, 98304));
  CHECK(hipMemset(counters, 0, 4096));
  it = 0;
  chain("no-wait chain (arrive only), 12 waves (D 3)", chain_kernel<12, 3, 0>, 768);
  CHECK(hipMemset(counters, 0, 4096));
  it = 0;
  chain("no-wait chain (arrive only), 12 waves (D 5)", chain_kernel<12, 5, 0>, 768);
  timeit("3 launches, ncu x 12 waves (D 5)", [&](int i) {
    const int s = i % ROT;
    for (int p = 0; p < NPH; ++p)
      hipLaunchKernelGGL((phase_kernel<12, 5>), dim3(ncu), dim3(768), 0, 0, sets[p][s], sl[p], sink);
  });
  return 0;
}
