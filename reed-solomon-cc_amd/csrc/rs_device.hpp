// rs_device.hpp — CDNA4 (gfx950) device primitives for the GF(2^16) additive FFT.
//
// Data in registers: a lane owns NV "dword pairs" of one 64-byte chunk column —
// lo dword j holds the low bytes of 4 symbols (chunk bytes [4j, 4j+4)), hi dword
// j their high bytes (chunk bytes [32+4j, 32+4j+4)) — the reference's chunk
// layout (Generic.zig:152-156) read straight from HBM, no transposition.
//
// Multiply by a constant (Generic.zig:275-298 `mul`): 6 bit-field selectors per
// dword pair, 12 v_perm_b32 table lookups (4 symbols each), 6 v_bitop3 XOR3.
// Twiddle tables (RsTab, 96 B) are wave-uniform: scalar-loaded from the plan.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

#include "rs_gf.hpp"

namespace rs {
namespace dev {

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// v_perm_b32: byte i of result = byte sel.byte[i] of the 8-byte value {hi_dw:lo_dw}
__device__ __forceinline__ uint32_t perm(uint32_t hi_dw, uint32_t lo_dw, uint32_t sel) {
  return __builtin_amdgcn_perm(hi_dw, lo_dw, sel);
}

template <int NV>
struct Sym {
  uint32_t l[NV];
  uint32_t h[NV];
};

// Uniform table view (held in SGPRs after a scalar load).
struct Tab {
  uint32_t lo[10];
  uint32_t hi[10];
  uint32_t flags;
};

// `t` must be a wave-uniform address into read-only plan memory. Reading it
// through the constant address space makes the compiler emit s_load_dwordx*
// so the table lives in SGPRs (a plain global pointer gives per-lane VMEM loads).
typedef const __attribute__((address_space(4))) RsTab *ConstTab;
__device__ __forceinline__ Tab load_tab(const RsTab *t) {
  ConstTab c = (ConstTab)(t);
  Tab r;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    r.lo[i] = c->lo[i];
    r.hi[i] = c->hi[i];
  }
  r.flags = c->flags;
  return r;
}

// product byte-planes of mul(y) for one dword pair, XORed into (xl, xh)
__device__ __forceinline__ void mul_acc1(uint32_t &xl, uint32_t &xh, uint32_t yl, uint32_t yh, const Tab &t) {
  const uint32_t a0 = yl & 0x07070707u, a1 = (yl >> 3) & 0x07070707u, a2 = (yl >> 6) & 0x03030303u;
  const uint32_t b0 = yh & 0x07070707u, b1 = (yh >> 3) & 0x07070707u, b2 = (yh >> 6) & 0x03030303u;
  uint32_t l = xor3(xl, perm(t.lo[1], t.lo[0], a0), perm(t.lo[3], t.lo[2], a1));
  uint32_t h = xor3(xh, perm(t.hi[1], t.hi[0], a0), perm(t.hi[3], t.hi[2], a1));
  l = xor3(l, perm(t.lo[4], t.lo[4], a2), perm(t.lo[6], t.lo[5], b0));
  h = xor3(h, perm(t.hi[4], t.hi[4], a2), perm(t.hi[6], t.hi[5], b0));
  xl = xor3(l, perm(t.lo[8], t.lo[7], b1), perm(t.lo[9], t.lo[9], b2));
  xh = xor3(h, perm(t.hi[8], t.hi[7], b1), perm(t.hi[9], t.hi[9], b2));
}

// Generic.zig:234-240 mulAdd: x ^= mul(y)
template <int NV>
__device__ __forceinline__ void mul_add(Sym<NV> &x, const Sym<NV> &y, const Tab &t) {
#pragma unroll
  for (int v = 0; v < NV; v++) mul_acc1(x.l[v], x.h[v], y.l[v], y.h[v], t);
}

// Generic.zig:220-231 mulScalar on one register slot: x = mul(x)
template <int NV>
__device__ __forceinline__ void mul_inplace(Sym<NV> &x, const Tab &t) {
#pragma unroll
  for (int v = 0; v < NV; v++) {
    uint32_t l = 0, h = 0;
    mul_acc1(l, h, x.l[v], x.h[v], t);
    x.l[v] = l;
    x.h[v] = h;
  }
}

template <int NV>
__device__ __forceinline__ void xor_into(Sym<NV> &a, const Sym<NV> &b) {
#pragma unroll
  for (int v = 0; v < NV; v++) {
    a.l[v] ^= b.l[v];
    a.h[v] ^= b.h[v];
  }
}

template <int NV>
__device__ __forceinline__ void zero(Sym<NV> &a) {
#pragma unroll
  for (int v = 0; v < NV; v++) a.l[v] = a.h[v] = 0;
}

// Generic.zig:149-169 fftPartial: x ^= mul(y); y ^= x   (XOR-only: y ^= x)
template <int NV>
__device__ __forceinline__ void fft_bf(Sym<NV> &x, Sym<NV> &y, const Tab &t) {
  if (!(t.flags & kTabXorOnly)) mul_add(x, y, t);
  xor_into(y, x);
}

// Generic.zig:171-192 ifftPartial: y ^= x; x ^= mul(y)   (XOR-only: y ^= x)
template <int NV>
__device__ __forceinline__ void ifft_bf(Sym<NV> &x, Sym<NV> &y, const Tab &t) {
  xor_into(y, x);
  if (!(t.flags & kTabXorOnly)) mul_add(x, y, t);
}

// ---- register-resident transforms over s[0..SIZE) (pos = 0), compile-time
// SIZE, run-time truncation. Table order = push_ifft_tabs / push_fft_tabs.

// Generic.zig:80-147
template <int SIZE, int NV>
__device__ __forceinline__ void ifft_regs(Sym<NV> *s, const RsTab *__restrict__ tabs, uint32_t trunc) {
  int ti = 0;
  int d = 1;
#pragma unroll
  for (int d4 = 4; d4 <= SIZE; d4 <<= 2) {
#pragma unroll
    for (int r = 0; r < SIZE; r += d4) {
      if (static_cast<uint32_t>(r) < trunc) {
        const Tab m01 = load_tab(tabs + ti), m02 = load_tab(tabs + ti + 1), m23 = load_tab(tabs + ti + 2);
#pragma unroll
        for (int i = r; i < r + d; i++) {
          ifft_bf(s[i], s[i + d], m01);
          ifft_bf(s[i + 2 * d], s[i + 3 * d], m23);
          ifft_bf(s[i], s[i + 2 * d], m02);
          ifft_bf(s[i + d], s[i + 3 * d], m02);
        }
      }
      ti += 3;
    }
    d = d4;
  }
  if (d < SIZE) {  // final odd layer, Generic.zig:131-146
    const Tab t = load_tab(tabs + ti);
#pragma unroll
    for (int i = 0; i < d; i++) ifft_bf(s[i], s[d + i], t);
  }
}

// Generic.zig:15-78
template <int SIZE, int NV>
__device__ __forceinline__ void fft_regs(Sym<NV> *s, const RsTab *__restrict__ tabs, uint32_t trunc) {
  int ti = 0;
  int d4 = SIZE;
#pragma unroll
  for (int d = SIZE >> 2; d != 0; d >>= 2) {
#pragma unroll
    for (int r = 0; r < SIZE; r += d4) {
      if (static_cast<uint32_t>(r) < trunc) {
        const Tab m01 = load_tab(tabs + ti), m02 = load_tab(tabs + ti + 1), m23 = load_tab(tabs + ti + 2);
#pragma unroll
        for (int i = r; i < r + d; i++) {
          fft_bf(s[i], s[i + 2 * d], m02);
          fft_bf(s[i + d], s[i + 3 * d], m02);
          fft_bf(s[i], s[i + d], m01);
          fft_bf(s[i + 2 * d], s[i + 3 * d], m23);
        }
      }
      ti += 3;
    }
    d4 = d;
  }
  if (d4 == 2) {  // radix-2 tail, Generic.zig:64-77
#pragma unroll
    for (int r = 0; r < SIZE; r += 2) {
      if (static_cast<uint32_t>(r) < trunc) {
        const Tab t = load_tab(tabs + ti + r / 2);
        fft_bf(s[r], s[r + 1], t);
      }
    }
  }
}

// ---- global-memory access for one lane's dword pairs -----------------------
template <int NV>
struct VecT;
template <>
struct VecT<1> {
  typedef uint32_t type;
};
template <>
struct VecT<2> {
  typedef uint32_t __attribute__((ext_vector_type(2))) type;
};
template <>
struct VecT<4> {
  typedef uint32_t __attribute__((ext_vector_type(4))) type;
};

// Two lane layouts for a lane's NV dword pairs (4*NV symbols):
//  * split  — lo dwords at p, hi dwords at p + 32 of one 64-B chunk; a wave
//             instruction touches half of every 64-B segment it spans.
//  * contig — a wave covers a region of 2 x 64*P bytes (P = 4*NV) with two loads
//             that are each fully contiguous: lanes 0-31 read lo pieces, lanes 32-63
//             the matching hi pieces; one v_permlane32_swap per dword then pairs every
//             lane's lo with its hi. p = the lane's first address, second at p + 64*P.
// Measured on MI355X (tools/hbm_probe.hip): contiguous wave accesses stream ~5% faster.
// `base` is wave-uniform (stripe/shard start) and `off` the lane's 32-bit offset,
// so the compiler can use the SGPR-base form of global_load/store (saddr + voffset).
// load_sym = load_sym_raw (issue the loads) + pair_halves (the contig swap, which
// must wait for them). Kernels loading several slots issue every raw load first and
// pair afterwards: a swap right behind its own load serialises one HBM round trip
// per slot (s_waitcnt vmcnt(0) before each v_permlane32_swap).
template <int NV>
__device__ __forceinline__ void load_sym_raw(Sym<NV> &s, const uint8_t *__restrict__ base, uint32_t off,
                                             bool contig) {
  typedef typename VecT<NV>::type V;
  const uint8_t *p = base + off;
  const V a = __builtin_nontemporal_load(reinterpret_cast<const V *>(p));
  const V b = __builtin_nontemporal_load(reinterpret_cast<const V *>(p + (contig ? 256 * NV : 32)));
  if constexpr (NV == 1) {
    s.l[0] = a;
    s.h[0] = b;
  } else {
#pragma unroll
    for (int v = 0; v < NV; v++) {
      s.l[v] = a[v];
      s.h[v] = b[v];
    }
  }
}

template <int NV>
__device__ __forceinline__ void pair_halves(Sym<NV> &s, bool contig) {
  if (contig) {
#pragma unroll
    for (int v = 0; v < NV; v++) {
      const auto r = __builtin_amdgcn_permlane32_swap(s.l[v], s.h[v], false, false);
      s.l[v] = r[0];
      s.h[v] = r[1];
    }
  }
}

template <int NV>
__device__ __forceinline__ void load_sym(Sym<NV> &s, const uint8_t *__restrict__ base, uint32_t off, bool contig) {
  load_sym_raw(s, base, off, contig);
  pair_halves(s, contig);
}

template <int NV>
__device__ __forceinline__ void store_sym(uint8_t *__restrict__ base, uint32_t off, const Sym<NV> &s, bool contig) {
  typedef typename VecT<NV>::type V;
  uint8_t *p = base + off;
  uint32_t l[NV], h[NV];
#pragma unroll
  for (int v = 0; v < NV; v++) {
    l[v] = s.l[v];
    h[v] = s.h[v];
  }
  if (contig) {
#pragma unroll
    for (int v = 0; v < NV; v++) {
      const auto r = __builtin_amdgcn_permlane32_swap(l[v], h[v], false, false);
      l[v] = r[0];
      h[v] = r[1];
    }
  }
  V a, b;
  if constexpr (NV == 1) {
    a = l[0];
    b = h[0];
  } else {
#pragma unroll
    for (int v = 0; v < NV; v++) {
      a[v] = l[v];
      b[v] = h[v];
    }
  }
  __builtin_nontemporal_store(a, reinterpret_cast<V *>(p));
  __builtin_nontemporal_store(b, reinterpret_cast<V *>(p + (contig ? 256 * NV : 32)));
}

// Byte offset of lane `lane` of wave `wave` (both within one stripe's shard) for
// the layouts above. contig needs shard_bytes % (512*NV) == 0 so every wave is
// whole (the swap needs all 64 lanes).
template <int NV>
__device__ __forceinline__ uint32_t lane_byte_offset(uint64_t wave, uint32_t lane, bool contig) {
  constexpr uint32_t P = 4 * NV, kPiecesPerHalf = 32 / P;
  if (contig) {
    const uint32_t ll = lane % 32;
    return static_cast<uint32_t>(wave * (128 * P) + ll / kPiecesPerHalf * 64 + (lane >= 32 ? 32 : 0) +
                                 ll % kPiecesPerHalf * P);
  }
  const uint64_t unit = wave * 64 + lane;
  return static_cast<uint32_t>(unit / (8 / NV) * 64 + unit % (8 / NV) * P);
}

}  // namespace dev
}  // namespace rs
