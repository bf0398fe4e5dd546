// c4_probe.hip — memory ceiling of the c4 traffic shape (RS(200,55), 256 KiB shards): the FFT
// kernels' unit is a 2 KiB slice of every shard of one stripe, one 8-wave workgroup per CU
// walking the units persistently; a wave reads its rows of the unit (two 1 KiB loads per row,
// raw buffer loads with the FFT kernels' nt policy) and writes its share of the m output rows
// (XOR of what it read: negligible ALU). Swept: workgroups per CU, rows in flight per wave,
// SEG bytes of each row per unit (2 / 4 / 8 KiB), nt on / off, interleaved / blocked unit walk. Build + run:
//   hipcc -O3 --offload-arch=gfx950 tools/c4_probe.hip -o tools/c4_probe && tools/c4_probe [stripes]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));

template <int K, int M, int NT, int RIF, int SEG, int BLK>
__global__ __launch_bounds__(512) void probe(const uint8_t *in, uint8_t *out, uint32_t sb, uint64_t n_units) {
  // SEG bytes of every row per unit (SEG / 1024 b128 loads per lane and row); BLK: workgroup b walks
  // units [b per, (b + 1) per) (a stripe's units in a row) instead of b, b + grid, ...
  constexpr uint32_t NL = SEG / 1024;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint32_t ups = sb / SEG;
  const uint64_t per = (n_units + gridDim.x - 1) / gridDim.x;
  const uint64_t u0 = BLK ? blockIdx.x * per : blockIdx.x, u1 = BLK ? (u0 + per < n_units ? u0 + per : n_units) : n_units;
  const uint64_t step = BLK ? 1 : gridDim.x;
  for (uint64_t u = u0; u < u1; u += step) {
    const uint64_t s = u / ups;
    const uint32_t uo = static_cast<uint32_t>(u - s * ups) * SEG + lane * 16u;
    const __amdgpu_buffer_rsrc_t R =
        __builtin_amdgcn_make_buffer_rsrc((void *)(in + s * K * sb), (short)0, (int)(K * sb), 0x00020000);
    const __amdgpu_buffer_rsrc_t O =
        __builtin_amdgcn_make_buffer_rsrc((void *)(out + s * M * sb), (short)0, (int)(M * sb), 0x00020000);
    u4 acc[NL] = {};
    // RIF rows' loads in flight per wave (unrolled groups: the loads of a group are issued
    // before any is consumed)
    for (uint32_t r0 = w; r0 < K; r0 += 8 * RIF) {
      u4 l[RIF][NL];
#pragma unroll
      for (int i = 0; i < RIF; i++) {
        const uint32_t r = r0 + 8u * i < K ? r0 + 8u * i : w;
#pragma unroll
        for (uint32_t q = 0; q < NL; q++) l[i][q] = __builtin_amdgcn_raw_buffer_load_b128(R, uo + q * 1024u, r * sb, NT);
      }
#pragma unroll
      for (int i = 0; i < RIF; i++)
        if (r0 + 8u * i < K)
#pragma unroll
          for (uint32_t q = 0; q < NL; q++) acc[q] ^= l[i][q];
    }
    for (uint32_t r = w; r < M; r += 8)
#pragma unroll
      for (uint32_t q = 0; q < NL; q++) __builtin_amdgcn_raw_buffer_store_b128(acc[q] + r, O, uo + q * 1024u, r * sb, NT);
  }
}

template <int K, int M, int NT, int RIF, int SEG, int BLK>
float run(const uint8_t *in, uint8_t *out, uint32_t sb, uint64_t n, int cus, int bpc, int reps) {
  const uint64_t units = n * (sb / SEG);
  const uint32_t grid = static_cast<uint32_t>(units < uint64_t(cus) * bpc ? units : uint64_t(cus) * bpc);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((probe<K, M, NT, RIF, SEG, BLK>), dim3(grid), dim3(512), 0, 0, in, out, sb, units);
  hipEventRecord(a);
  for (int r = 0; r < reps; r++)
    hipLaunchKernelGGL((probe<K, M, NT, RIF, SEG, BLK>), dim3(grid), dim3(512), 0, 0, in, out, sb, units);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

template <int NT, int SEG, int BLK>
void sweep(const uint8_t *in, uint8_t *out, uint32_t sb, uint64_t n, int cus) {
  const double enc = double(n) * (200 + 55) * sb;
  for (int bpc : {1, 2}) {
    for (int rep = 0; rep < 2; rep++) {
      const float t1 = run<200, 55, NT, 1, SEG, BLK>(in, out, sb, n, cus, bpc, 10);
      const float t4 = run<200, 55, NT, 4, SEG, BLK>(in, out, sb, n, cus, bpc, 10);
      const float t8 = run<200, 55, NT, 8, SEG, BLK>(in, out, sb, n, cus, bpc, 10);
      std::printf("{\"shape\": \"c4 RS(200,55) 256 KiB x %llu\", \"seg_bytes\": %d, \"nt\": %d, \"blocked\": %d, "
                  "\"wg_per_cu\": %d, \"rif1_ms\": %.3f, \"rif4_ms\": %.3f, \"rif8_ms\": %.3f, \"best_TBps\": %.3f, "
                  "\"best_frac\": %.4f}\n",
                  (unsigned long long)n, SEG, NT ? 1 : 0, BLK, bpc, t1, t4, t8,
                  enc / std::min(t1, std::min(t4, t8)) / 1e9, enc / std::min(t1, std::min(t4, t8)) / 1e9 / 8000.0);
      std::fflush(stdout);
    }
  }
}

int main(int argc, char **argv) {
  const uint32_t sb = 256u << 10;
  const uint64_t n = argc > 1 ? atoll(argv[1]) : 256;
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint8_t *in, *out;
  if (hipMalloc(&in, n * 200 * sb) || hipMalloc(&out, n * 55 * sb)) return 1;
  hipMemset(in, 0x5a, n * 200 * sb);
  // per-row segment 2 / 4 / 8 KiB x nt on / off x interleaved / blocked walk
  sweep<2, 2048, 0>(in, out, sb, n, cus);
  sweep<0, 2048, 0>(in, out, sb, n, cus);
  sweep<2, 2048, 1>(in, out, sb, n, cus);
  sweep<2, 4096, 0>(in, out, sb, n, cus);
  sweep<0, 4096, 0>(in, out, sb, n, cus);
  sweep<2, 4096, 1>(in, out, sb, n, cus);
  sweep<2, 8192, 0>(in, out, sb, n, cus);
  sweep<0, 8192, 0>(in, out, sb, n, cus);
  return 0;
}
