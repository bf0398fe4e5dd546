// rs_xform.hpp — the column transforms' device primitives shared by the precompiled kernels
// (rs_kernels.hip):
// Generic.zig:15-147 on a register set of N positions (ifft_sub / fft_sub, wave-uniform
// twiddle tables in SGPRs), the opaque-value helpers that keep table addresses from being
// hoisted out of loops, and the buffer resources of shard rows.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "rs_device.hpp"

namespace rs {
namespace dev {

__device__ __forceinline__ uint32_t log2_u64(uint64_t x) { return 63u - static_cast<uint32_t>(__builtin_clzll(x)); }

// A butterfly group's three twiddle tables are 63 SGPRs. A scheduling barrier after each group
// keeps the scheduler from lifting the next groups' table loads above it; on its own it did not
// change the phase kernels' SGPR spills (those came from loop-invariant hoisting, see opq), so
// it is kept as the per-group boundary the opaque tables below rely on.
__device__ __forceinline__ void group_fence() { __builtin_amdgcn_sched_barrier(0); }
// Values the compiler cannot prove loop-invariant (see opq(PhaseArgs)): plus a zero that a
// volatile SALU move produces in place, so nothing derived from them is hoisted out of the
// loop that calls this. (A readfirstlane round trip did the same but read an SGPR copy the
// compiler had made in VGPRs under a narrower EXEC: garbage table addresses in partial waves.)
__device__ __forceinline__ uint32_t vzero() {
  uint32_t z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return z;
}
template <class T>
__device__ __forceinline__ T *opq(T *p) {
  return p + vzero();
}
__device__ __forceinline__ uint64_t opqu(uint64_t v) { return v + vzero(); }
__device__ __forceinline__ uint32_t opqu(uint32_t v) { return v + vzero(); }

// Generic.zig:80-147 on one position set (ti: table index of the phase's first layer). The
// group table offsets derive from opaque copies of ti / blk / dlo_log: computed where each
// group runs, not hoisted out of the callers' loops and held (spilled) across them.
template <int N, int NV>
__device__ __forceinline__ void ifft_sub(Sym<NV> *s, const RsTab *__restrict__ tabs, uint64_t ti, uint64_t size,
                                         uint64_t rmax, uint64_t blk, uint32_t dlo_log) {
  ti = opqu(ti);
  blk = opqu(blk);
  dlo_log = opqu(dlo_log);
  int jd = 1;
#pragma unroll
  for (int jd4 = 4; jd4 <= N; jd4 <<= 2) {
    const uint32_t lg4 = static_cast<uint32_t>(__builtin_ctz(jd4)) + dlo_log;
#pragma unroll
    for (int jr = 0; jr < N; jr += jd4) {
      const uint64_t r = blk + (static_cast<uint64_t>(jr) << dlo_log);
      if (r < rmax) {
        const RsTab *g = tabs + ti + 3 * (r >> lg4);
        const Tab m01 = dev::load_tab(g), m02 = dev::load_tab(g + 1), m23 = dev::load_tab(g + 2);
#pragma unroll
        for (int i = jr; i < jr + jd; i++) {
          dev::ifft_bf(s[i], s[i + jd], m01);
          dev::ifft_bf(s[i + 2 * jd], s[i + 3 * jd], m23);
          dev::ifft_bf(s[i], s[i + 2 * jd], m02);
          dev::ifft_bf(s[i + jd], s[i + 3 * jd], m02);
        }
      }
      group_fence();
    }
    ti += 3 * (size >> lg4);
    jd = jd4;
  }
  if (jd < N) {  // the final odd layer (distance size/2): one table, no truncation
    const Tab t = dev::load_tab(tabs + ti);
#pragma unroll
    for (int i = 0; i < jd; i++) dev::ifft_bf(s[i], s[jd + i], t);
  }
}

// Generic.zig:15-78 on one position set
template <int N, int NV>
__device__ __forceinline__ void fft_sub(Sym<NV> *s, const RsTab *__restrict__ tabs, uint64_t ti, uint64_t size,
                                        uint64_t rmax, uint64_t blk, uint32_t dlo_log) {
  ti = opqu(ti);
  blk = opqu(blk);
  dlo_log = opqu(dlo_log);
  int jd4 = N;
#pragma unroll
  for (int jd = N >> 2; jd != 0; jd >>= 2) {
    const uint32_t lg4 = static_cast<uint32_t>(__builtin_ctz(jd4)) + dlo_log;
#pragma unroll
    for (int jr = 0; jr < N; jr += jd4) {
      const uint64_t r = blk + (static_cast<uint64_t>(jr) << dlo_log);
      if (r < rmax) {
        const RsTab *g = tabs + ti + 3 * (r >> lg4);
        const Tab m01 = dev::load_tab(g), m02 = dev::load_tab(g + 1), m23 = dev::load_tab(g + 2);
#pragma unroll
        for (int i = jr; i < jr + jd; i++) {
          dev::fft_bf(s[i], s[i + 2 * jd], m02);
          dev::fft_bf(s[i + jd], s[i + 3 * jd], m02);
          dev::fft_bf(s[i], s[i + jd], m01);
          dev::fft_bf(s[i + 2 * jd], s[i + 3 * jd], m23);
        }
      }
      group_fence();
    }
    ti += 3 * (size >> lg4);
    jd4 = jd;
  }
  if (jd4 == 2) {  // radix-2 tail (distance 1, so dlo == 1): a table per pair
#pragma unroll
    for (int jr = 0; jr < N; jr += 2) {
      const uint64_t r = blk + static_cast<uint64_t>(jr);
      if (r < rmax) {
        const Tab t = dev::load_tab(tabs + ti + r / 2);
        dev::fft_bf(s[jr], s[jr + 1], t);
      }
      group_fence();
    }
  }
}

// a lane's dword pair(s) at row + off (split layout) through a buffer resource whose base
// is the wave-uniform row address: the loads keep the SGPR base + 32-bit lane offset form
// (a plain pointer walk gets its per-lane 64-bit address math hoisted into VGPRs)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const uint8_t *row) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(row), static_cast<short>(0), 0x7FFFFFFF, 0x00020000);
}
// a resource with no records: loads through it read zero, stores through it are dropped
__device__ __forceinline__ __amdgpu_buffer_rsrc_t zero_rsrc() {
  return __builtin_amdgcn_make_buffer_rsrc(nullptr, static_cast<short>(0), 0, 0x00020000);
}
}  // namespace dev
}  // namespace rs
