// c4_probe.hip — memory ceiling of the c4 traffic shape (RS(200,55), 256 KiB shards): the FFT
// kernels' unit is a 2 KiB slice of every shard of one stripe, one 8-wave workgroup per CU
// walking the units persistently; a wave reads its rows of the unit (two 1 KiB loads per row,
// raw buffer loads with the FFT kernels' nt policy) and writes its share of the m output rows
// (XOR of what it read: negligible ALU). BPC workgroups per CU. Build + run:
//   hipcc -O3 --offload-arch=gfx950 tools/c4_probe.hip -o tools/c4_probe && tools/c4_probe [stripes]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

template <int K, int M, int NT, int RIF>
__global__ __launch_bounds__(512) void probe(const uint8_t *in, uint8_t *out, uint32_t sb, uint64_t n_units) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint32_t ups = sb / 2048u;
  for (uint64_t u = blockIdx.x; u < n_units; u += gridDim.x) {
    const uint64_t s = u / ups;
    const uint32_t uo = static_cast<uint32_t>(u - s * ups) * 2048u + lane * 16u;
    const __amdgpu_buffer_rsrc_t R =
        __builtin_amdgcn_make_buffer_rsrc((void *)(in + s * K * sb), (short)0, (int)(K * sb), 0x00020000);
    const __amdgpu_buffer_rsrc_t O =
        __builtin_amdgcn_make_buffer_rsrc((void *)(out + s * M * sb), (short)0, (int)(M * sb), 0x00020000);
    u4 a = {0, 0, 0, 0}, b = {0, 0, 0, 0};
    // RIF rows' loads in flight per wave (unrolled groups: the loads of a group are issued
    // before any is consumed)
    for (uint32_t r0 = w; r0 < K; r0 += 8 * RIF) {
      u4 la[RIF], lb[RIF];
#pragma unroll
      for (int i = 0; i < RIF; i++) {
        const uint32_t r = r0 + 8u * i < K ? r0 + 8u * i : w;
        la[i] = __builtin_amdgcn_raw_buffer_load_b128(R, uo, r * sb, NT);
        lb[i] = __builtin_amdgcn_raw_buffer_load_b128(R, uo + 1024u, r * sb, NT);
      }
#pragma unroll
      for (int i = 0; i < RIF; i++)
        if (r0 + 8u * i < K) a ^= la[i], b ^= lb[i];
    }
    for (uint32_t r = w; r < M; r += 8) {
      __builtin_amdgcn_raw_buffer_store_b128(a + r, O, uo, r * sb, NT);
      __builtin_amdgcn_raw_buffer_store_b128(b + r, O, uo + 1024u, r * sb, NT);
    }
  }
}

template <int K, int M, int NT, int RIF>
float run(const uint8_t *in, uint8_t *out, uint32_t sb, uint64_t n, int cus, int bpc, int reps) {
  const uint64_t units = n * (sb / 2048);
  const uint32_t grid = static_cast<uint32_t>(units < uint64_t(cus) * bpc ? units : uint64_t(cus) * bpc);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((probe<K, M, NT, RIF>), dim3(grid), dim3(512), 0, 0, in, out, sb, units);
  hipEventRecord(a);
  for (int r = 0; r < reps; r++) hipLaunchKernelGGL((probe<K, M, NT, RIF>), dim3(grid), dim3(512), 0, 0, in, out, sb, units);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main(int argc, char **argv) {
  const uint32_t sb = 256u << 10;
  const uint64_t n = argc > 1 ? atoll(argv[1]) : 256;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint8_t *in, *out;
  if (hipMalloc(&in, n * 200 * sb) || hipMalloc(&out, n * 55 * sb)) return 1;
  hipMemset(in, 0x5a, n * 200 * sb);
  const double enc = double(n) * (200 + 55) * sb, dec = double(n) * (145 + 55 + 55) * sb;
  for (int bpc : {1, 2}) {
    for (int rep = 0; rep < 2; rep++) {
      const float t1 = run<200, 55, 2, 1>(in, out, sb, n, cus, bpc, 10), t4 = run<200, 55, 2, 4>(in, out, sb, n, cus, bpc, 10);
      const float t8 = run<200, 55, 2, 8>(in, out, sb, n, cus, bpc, 10), t25 = run<200, 55, 2, 25>(in, out, sb, n, cus, bpc, 10);
      std::printf("{\"shape\": \"c4 RS(200,55) 256 KiB x %llu, 2 KiB units, 8-wave WGs, nt\", \"wg_per_cu\": %d, "
                  "\"rows_in_flight_1_ms\": %.3f, \"rif4_ms\": %.3f, \"rif8_ms\": %.3f, \"rif25_ms\": %.3f, "
                  "\"best_TBps\": %.3f}\n",
                  (unsigned long long)n, bpc, t1, t4, t8, t25,
                  enc / std::min(std::min(t1, t4), std::min(t8, t25)) / 1e9);
    }
  }
  (void)dec;
  return 0;
}
