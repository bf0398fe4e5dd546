// hbm_probe.hip — memory-system ceiling for the codec's traffic shape on MI355X.
// Reads k shards and writes m "parity" shards per stripe ([stripe][shard][sb]),
// parity = XOR of the inputs (negligible ALU), with the access patterns the
// codec kernels can use:
//   split   : lane pair per 64-B chunk; 16-B loads of the lo half and of the hi half
//             (what k_encode_reg<.,4> does)
//   contig  : each wave instruction covers 1 KiB contiguously (16 B per lane)
// x {default, nontemporal} cache policy. Build + run:
//   hipcc -O3 --offload-arch=gfx950 tools/hbm_probe.hip -o tools/hbm_probe && tools/hbm_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ u4 ld(const u4 *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u4 *p, u4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int K, int M, bool SPLIT, bool NT>
__global__ __launch_bounds__(256) void probe(const uint8_t *in, uint8_t *out, uint64_t sb, uint64_t n) {
  const uint64_t unit = static_cast<uint64_t>(blockIdx.x) * 256 + threadIdx.x;  // 32 B per lane
  if (unit * 32 >= sb) return;
  uint64_t o0, o1;
  if (SPLIT) {  // lane pair per chunk: lo[16u..] and hi[32+16u..]
    o0 = unit / 2 * 64 + (unit % 2) * 16;
    o1 = o0 + 32;
  } else {  // two contiguous 1 KiB sweeps per wave
    const uint64_t w = unit / 64, l = unit % 64;
    o0 = w * 2048 + l * 16;
    o1 = o0 + 1024;
  }
  for (uint64_t s = blockIdx.y; s < n; s += gridDim.y) {
    const uint8_t *src = in + s * K * sb;
    u4 a0 = {0, 0, 0, 0}, a1 = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < K; i++) {
      a0 ^= ld<NT>(reinterpret_cast<const u4 *>(src + i * sb + o0));
      a1 ^= ld<NT>(reinterpret_cast<const u4 *>(src + i * sb + o1));
    }
    uint8_t *dst = out + s * M * sb;
#pragma unroll
    for (int j = 0; j < M; j++) {
      st<NT>(reinterpret_cast<u4 *>(dst + j * sb + o0), a0 + j);
      st<NT>(reinterpret_cast<u4 *>(dst + j * sb + o1), a1 + j);
    }
  }
}

// unit4k: a wave covers a 4 KiB unit of every shard, four 16-B loads per lane 1 KiB apart
// (the network kernels' pattern); one wave per unit, 4 waves per workgroup
template <int K, int M, bool NT>
__global__ __launch_bounds__(256) void probe4k(const uint8_t *in, uint8_t *out, uint64_t sb, uint64_t n) {
  const uint64_t units = sb / 4096, lane = threadIdx.x & 63;
  const uint64_t u = static_cast<uint64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (u >= units) return;
  for (uint64_t s = blockIdx.y; s < n; s += gridDim.y) {
    const uint8_t *src = in + s * K * sb + u * 4096 + lane * 16;
    u4 a[4] = {};
#pragma unroll
    for (int i = 0; i < K; i++)
#pragma unroll
      for (int q = 0; q < 4; q++) a[q] ^= ld<NT>(reinterpret_cast<const u4 *>(src + i * sb + q * 1024));
    uint8_t *dst = out + s * M * sb + u * 4096 + lane * 16;
    if (M == 0) {  // read-only shape: every loaded dword decides a (never taken) store
      const u4 t = a[0] ^ a[1] ^ a[2] ^ a[3];
      if ((t.x ^ t.y ^ t.z ^ t.w) == 0x9e3779b9u) st<NT>(reinterpret_cast<u4 *>(out + lane * 16), t);
    }
#pragma unroll
    for (int j = 0; j < M; j++)
#pragma unroll
      for (int q = 0; q < 4; q++) st<NT>(reinterpret_cast<u4 *>(dst + j * sb + q * 1024), a[q] + j);
  }
}

template <int K, int M, bool NT>
float run4k(const uint8_t *in, uint8_t *out, uint64_t sb, uint64_t n, int reps) {
  dim3 grid((sb / 4096 + 3) / 4, n < 65535 ? n : 65535);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((probe4k<K, M, NT>), grid, dim3(256), 0, 0, in, out, sb, n);
  hipEventRecord(a);
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL((probe4k<K, M, NT>), grid, dim3(256), 0, 0, in, out, sb, n);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

template <int K, int M, bool SPLIT, bool NT>
float run(const uint8_t *in, uint8_t *out, uint64_t sb, uint64_t n, int reps) {
  dim3 grid((sb / 32 + 255) / 256, n < 65535 ? n : 65535);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((probe<K, M, SPLIT, NT>), grid, dim3(256), 0, 0, in, out, sb, n);
  hipEventRecord(a);
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL((probe<K, M, SPLIT, NT>), grid, dim3(256), 0, 0, in, out, sb, n);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main(int argc, char **argv) {
  const uint64_t sb = 1 << 20, n = argc > 1 ? atoll(argv[1]) : 1024;
  uint8_t *in, *out;
  if (hipMalloc(&in, n * 10 * sb) || hipMalloc(&out, n * 4 * sb)) return 1;
  hipMemset(in, 1, n * 10 * sb);
  const double bytes = 14.0 * sb * n;
  struct V {
    const char *name;
    float (*f)(const uint8_t *, uint8_t *, uint64_t, uint64_t, int);
  } vs[] = {{"split  default", run<10, 4, true, false>},
            {"split  nt     ", run<10, 4, true, true>},
            {"contig default", run<10, 4, false, false>},
            {"contig nt     ", run<10, 4, false, true>},
            {"unit4k default", run4k<10, 4, false>},
            {"unit4k nt     ", run4k<10, 4, true>}};
  struct V2 {
    const char *name;
    float (*f)(const uint8_t *, uint8_t *, uint64_t, uint64_t, int);
  } shapes[] = {{"unit4k nt 14 read / 0 write", run4k<14, 0, true>},
                {"unit4k nt 7 read / 7 write ", run4k<7, 7, true>}};
  for (int round = 0; round < 2; round++)
    for (auto &v : shapes) {
      const float ms = v.f(in, out, sb, n / 2, 5);  // n/2 stripes of 14 shards fit both buffers
      printf("{\"variant\": \"%s\", \"round\": %d, \"ms\": %.3f, \"TBps\": %.3f}\n", v.name, round, ms,
             bytes / 2 / ms / 1e9);
    }
  for (int round = 0; round < 3; round++)
    for (auto &v : vs) {
      const float ms = v.f(in, out, sb, n, 5);
      printf("{\"variant\": \"%s\", \"round\": %d, \"ms\": %.3f, \"TBps\": %.3f}\n", v.name, round, ms,
             bytes / ms / 1e9);
    }
  return 0;
}
