// valu_probe.hip — issue cost of the codec's VALU instructions on MI355X.
// Each lane runs 8 independent dependency chains of one instruction form; the
// cycles per wave-instruction per SIMD come from s_memtime deltas (shader clock)
// and from the event-timed wall clock. Build + run:
//   hipcc -O3 --offload-arch=gfx950 tools/valu_probe.hip -o tools/valu_probe && tools/valu_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define OPS8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

enum Op { kPermVVV, kPermSVV, kBitop3, kXor, kXor3, kAnd, kMovS, kLshr, kAndOr, kBfe, kBitop3S, kBitop3Dep1,
          kBitop3Dep2, kNumOps };
static const char *kNames[] = {"v_perm_b32 v,v,v", "v_perm_b32 s,v,v", "v_bitop3_b32 v,v,v", "v_xor_b32",
                               "v_or3_b32",        "v_and_b32",        "v_mov_b32 v,s",      "v_lshrrev_b32",
                               "v_and_or_b32",     "v_bfe_u32",        "v_bitop3_b32 v,v,s", "bitop3 1 chain",
                               "bitop3 2 chains"};

template <int OP>
__global__ __launch_bounds__(256) void probe(uint32_t *out, uint64_t *cyc, uint32_t iters, uint32_t sval) {
  uint32_t x[8];
  const uint32_t t = threadIdx.x;
#pragma unroll
  for (int c = 0; c < 8; c++) x[c] = t * 2654435761u + c;
  uint32_t a = t ^ 0x1234567u, sel = 0x03020100u + (t & 0x04040404u);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
#define STEP(c)                                                                                            \
  if constexpr (OP == kPermVVV) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(x[c]) : "v"(a), "v"(sel)); \
  if constexpr (OP == kPermSVV) asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(x[c]) : "s"(sval), "v"(sel)); \
  if constexpr (OP == kBitop3) asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0x96" : "+v"(x[c]) : "v"(a), "v"(sel)); \
  if constexpr (OP == kXor) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x[c]) : "v"(a));                    \
  if constexpr (OP == kXor3) asm volatile("v_or3_b32 %0, %1, %0, %2" : "+v"(x[c]) : "v"(a), "v"(sel));    \
  if constexpr (OP == kAnd) asm volatile("v_and_b32 %0, %1, %0" : "+v"(x[c]) : "v"(a));                    \
  if constexpr (OP == kMovS) asm volatile("v_mov_b32 %0, %1" : "=v"(x[c]) : "s"(sval + c));                \
  if constexpr (OP == kLshr) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(x[c]));                          \
  if constexpr (OP == kAndOr) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(a), "v"(sel)); \
  if constexpr (OP == kBfe) asm volatile("v_bfe_u32 %0, %0, 3, 8" : "+v"(x[c]));                           \
  if constexpr (OP == kBitop3S) asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0x96" : "+v"(x[c]) : "v"(a), "s"(sval)); \
  if constexpr (OP == kBitop3Dep1) asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0x96" : "+v"(x[0]) : "v"(a), "v"(sel)); \
  if constexpr (OP == kBitop3Dep2) asm volatile("v_bitop3_b32 %0, %1, %0, %2 bitop3:0x96" : "+v"(x[c & 1]) : "v"(a), "v"(sel));
      OPS8(STEP)
#undef STEP
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  uint32_t r = 0;
#pragma unroll
  for (int c = 0; c < 8; c++) r ^= x[c];
  out[blockIdx.x * 256 + t] = r;
  if (t % 64 == 0) cyc[blockIdx.x * 4 + t / 64] = t1 - t0;
}

template <int OP>
void run(int blocks, uint32_t iters, uint32_t *out, uint64_t *cyc) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters, 0x01234567u);
  hipEventRecord(a);
  hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, out, cyc, iters, 0x01234567u);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  std::vector<uint64_t> c(blocks * 4);
  hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
  double mean = 0;
  for (auto v : c) mean += v;
  mean /= c.size();
  const double waves_per_simd = blocks * 4.0 / (256 * 4);
  const double winst = 32.0 * iters;  // wave-instructions per wave
  // per-wave cycles / instructions = cycles per instruction seen by one wave;
  // divided by waves sharing the SIMD = SIMD cycles per wave-instruction
  printf("%-22s waves/SIMD %4.1f  memtime-cyc/inst/SIMD %6.2f  wall %8.3f ms  (%.2f Ginst/s chip)\n", kNames[OP],
         waves_per_simd, mean / winst / waves_per_simd, ms, blocks * 4.0 * winst / ms / 1e6);
}

int main(int argc, char **argv) {
  const uint32_t iters = argc > 1 ? atoi(argv[1]) : 2000;
  uint32_t *out;
  uint64_t *cyc;
  hipMalloc(&out, 8192 * 256 * 4);
  hipMalloc(&cyc, 8192 * 4 * 8);
  for (int wps : {1, 2, 4, 8}) {
    const int blocks = 256 * wps;  // 4 waves per block, one per SIMD
    run<kPermVVV>(blocks, iters, out, cyc);
    run<kPermSVV>(blocks, iters, out, cyc);
    run<kBitop3>(blocks, iters, out, cyc);
    run<kXor>(blocks, iters, out, cyc);
    run<kXor3>(blocks, iters, out, cyc);
    run<kAnd>(blocks, iters, out, cyc);
    run<kMovS>(blocks, iters, out, cyc);
    run<kLshr>(blocks, iters, out, cyc);
    run<kAndOr>(blocks, iters, out, cyc);
    run<kBfe>(blocks, iters, out, cyc);
    run<kBitop3S>(blocks, iters, out, cyc);
    run<kBitop3Dep1>(blocks, iters, out, cyc);
    run<kBitop3Dep2>(blocks, iters, out, cyc);
  }
  return 0;
}
