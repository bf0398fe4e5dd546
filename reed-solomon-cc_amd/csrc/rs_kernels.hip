// rs_kernels.hip — HIP kernels for gfx950 (MI355X): Reed-Solomon encode and
// reconstruct over GF(2^16) with the additive FFT of usebeforefree/reed-solomon-cc.
//
// Parallelisation: every 64-byte chunk column of a stripe is an
// independent code, so a lane owns NV dword pairs (4*NV symbols) of one column
// and runs the WHOLE codec for it — no cross-lane exchange, no barriers, no LDS.
// Grid: x = column units of one stripe (256 lanes per block), y = stripes.
//
//  * k_encode_reg<C, NV>: fused encode, the chunk-sized transforms in VGPRs.
//    HBM traffic = k shards read + m shards written per stripe (the minimum).
//    Mirrors Encoder.encode (root.zig:136-173).
//  * k_decode_reg<W, NV>: fused reconstruct, the W-point transforms in VGPRs.
//    Reads the k+m-e received shards it needs, writes the e restored ones.
//    Mirrors Decoder.decode (root.zig:268-335).
//  * k_encode_generic / launch_decode_generic: the same codec for any (k, m) through
//    a global scratch work buffer [stripe][W][shard_bytes] (the reference's Shards
//    layout, root.zig:350-395); the decode as a sequence of launches whose grid spans
//    the transform's positions (k_dec_gather, k_phase, k_dec_deriv, k_dec_scatter).
//  * k_engine_transform / k_mul_scalar: the Engine seam (Generic.zig) as test shims.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rs_device.hpp"
#include "rs_internal.hpp"
#include "rs_xform.hpp"

namespace rs {
namespace {

using dev::Sym;
using dev::Tab;
using dev::fft_sub;
using dev::group_fence;
using dev::ifft_sub;
using dev::log2_u64;
using dev::opq;
using dev::opqu;
using dev::row_rsrc;
using dev::vzero;
using dev::zero_rsrc;

constexpr int kBlock = 256;

__host__ __device__ constexpr int ifft_tabs_ce(int size) {
  int n = 0, d = 1, d4 = 4;
  for (; d4 <= size; d = d4, d4 <<= 2) n += 3 * (size / d4);
  return n + (d < size ? 1 : 0);
}

// byte offset of this lane's data inside a shard (dev::lane_byte_offset); false
// if the lane's unit is past the shard end (whole waves, see the layouts).
template <int NV>
__device__ __forceinline__ bool lane_offset(uint64_t shard_bytes, bool contig, uint32_t &off) {
  const uint64_t unit = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  if (unit >= shard_bytes / 64 * (8 / NV)) return false;
  off = dev::lane_byte_offset<NV>(unit / 64, static_cast<uint32_t>(unit % 64), contig);
  return true;
}

// Encode of a partial data set (reconstruct by syndromes, rs_capi.cpp): data
// shard `idx` flagged in the skip bitmask is read as zeros (never touched).
__device__ __forceinline__ bool skipped(const EncodeArgs &a, uint32_t idx) {
  typedef const __attribute__((address_space(4))) uint32_t *CU;
  return a.skip && ((((CU)(a.skip))[idx >> 5] >> (idx & 31)) & 1u);
}

// ============================================================ fused encode
template <int C, int NV>
__global__ __launch_bounds__(kBlock) void k_encode_reg(EncodeArgs a) {
  uint32_t off;
  if (!lane_offset<NV>(a.shard_bytes, a.contig, off)) return;
  constexpr int TI = ifft_tabs_ce(C);
  const uint64_t sb = a.shard_bytes;
  {  // one stripe per blockIdx.y (launches are split at 65535 stripes)
    const uint64_t s = blockIdx.y;
    const uint8_t *src = a.data + s * a.data_stripe_stride;
    Sym<NV> acc[C];
    // first chunk: root.zig:143-146
#pragma unroll
    for (int p = 0; p < C; p++) {
      if (static_cast<uint32_t>(p) < a.trunc_first && !skipped(a, p))
        dev::load_sym_raw(acc[p], src + p * sb, off, a.contig);
      else dev::zero(acc[p]);
    }
#pragma unroll
    for (int p = 0; p < C; p++) dev::pair_halves(acc[p], a.contig);
    dev::ifft_regs<C>(acc, a.tabs, a.trunc_first);
    // further chunks, IFFT + XOR-fold: root.zig:148-167
    for (uint32_t j = 1; j < a.n_chunks; j++) {
      const uint32_t t = (j + 1 == a.n_chunks) ? a.trunc_last : static_cast<uint32_t>(C);
      const uint8_t *cs = src + static_cast<uint64_t>(j) * C * sb;
      Sym<NV> cur[C];
#pragma unroll
      for (int p = 0; p < C; p++) {
        if (static_cast<uint32_t>(p) < t && !skipped(a, j * C + p)) dev::load_sym_raw(cur[p], cs + p * sb, off, a.contig);
        else dev::zero(cur[p]);
      }
#pragma unroll
      for (int p = 0; p < C; p++) dev::pair_halves(cur[p], a.contig);
      const RsTab *tj = a.tabs + j * TI;
      asm volatile("" : "+s"(tj));  // opaque base: no per-group pointer IVs (SGPR spills)
      dev::ifft_regs<C>(cur, tj, t);
#pragma unroll
      for (int p = 0; p < C; p++) dev::xor_into(acc[p], cur[p]);
    }
    // root.zig:169
    dev::fft_regs<C>(acc, a.tabs + a.n_chunks * TI, a.m);
    uint8_t *dst = a.parity + s * a.parity_stripe_stride;
#pragma unroll
    for (int p = 0; p < C; p++)
      if (static_cast<uint32_t>(p) < a.m) dev::store_sym(dst + p * sb, off, acc[p], a.contig);
  }
}

// ======================================================= fused reconstruct
// root.zig:309-315 formal derivative over W register slots
template <int W, int NV>
__device__ __forceinline__ void derivative_regs(Sym<NV> *w) {
#pragma unroll
  for (int i = 1; i < W; i++) {
    const int width = i & -i;
#pragma unroll
    for (int j = 0; j < width; j++) dev::xor_into(w[i - width + j], w[i + j]);
  }
}

template <int W, int NV>
__global__ __launch_bounds__(kBlock) void k_decode_reg(DecodeArgs a) {
  uint32_t off;
  if (!lane_offset<NV>(a.shard_bytes, a.contig, off)) return;
  const uint64_t sb = a.shard_bytes;
  {  // one stripe per blockIdx.y (launches are split at 65535 stripes)
    const uint64_t s = blockIdx.y;
    const uint8_t *orig = a.orig + s * a.orig_stripe_stride;
    const uint8_t *rec = a.rec + s * a.rec_stripe_stride;
    // shared plan, or this stripe's own (per-stripe erasure patterns)
    const RsTab *tab_pre = a.tab_pre + s * a.pattern_stride, *tab_post = a.tab_post + s * a.pattern_stride;
    const int32_t *pos_src = a.pos_src + s * a.pattern_stride, *pos_dst = a.pos_dst + s * a.pattern_stride;
    Sym<NV> w[W];
    // erasure masks on received shards, zero elsewhere: root.zig:291-303
#pragma unroll
    for (int p = 0; p < W; p++) {
      const int32_t src = ((const __attribute__((address_space(4))) int32_t *)pos_src)[p];
      if (src >= 0) {
        const uint8_t *base = (src & kSrcRecovery) ? rec : orig;
        dev::load_sym_raw(w[p], base + static_cast<uint64_t>(src & kSrcIndexMask) * sb, off, a.contig);
      } else {
        dev::zero(w[p]);
      }
    }
#pragma unroll
    for (int p = 0; p < W; p++) {  // all loads in flight before the first swap waits
      if (((const __attribute__((address_space(4))) int32_t *)pos_src)[p] >= 0) {
        dev::pair_halves(w[p], a.contig);
        dev::mul_inplace(w[p], dev::load_tab(tab_pre + p));
      }
    }
    dev::ifft_regs<W>(w, a.tab_ifft, a.trunc);  // root.zig:306
    derivative_regs<W>(w);                      // root.zig:309-315
    dev::fft_regs<W>(w, a.tab_fft, a.trunc_fft ? a.trunc_fft : a.trunc);  // root.zig:318
    uint8_t *out = a.out + s * a.out_stripe_stride;
#pragma unroll
    for (int p = 0; p < W; p++) {  // root.zig:321-326
      const int32_t dst = ((const __attribute__((address_space(4))) int32_t *)pos_dst)[p];
      if (dst >= 0) {
        dev::mul_inplace(w[p], dev::load_tab(tab_post + p));
        dev::store_sym(out + static_cast<uint64_t>(dst) * sb, off, w[p], a.contig);
      }
    }
  }
}

// ============================================ wave-split encode, chunk = 64
// For m in 33..64 the 64-point chunk transforms do not fit one lane's VGPRs.
// Four waves share the SAME 64 column units (lanes) and split the positions:
// layout A — wave w holds positions 16w+j (radix-4 stages on bits (0,1), (2,3)
// are wave-local); layout B — wave w holds positions i + 4w + 16q (stage on
// bits (4,5) wave-local). A <-> B is one LDS transpose per chunk. Every twiddle
// a wave needs is still wave-uniform (its group base depends only on w), so
// tables stay in SGPRs. Mirrors Encoder.encode (root.zig:136-173).
template <int NV>
struct LdsSym {
  uint32_t v[2 * NV];
};

template <int NV>
__device__ __forceinline__ void lds_put(LdsSym<NV> *row, uint32_t lane, const Sym<NV> &x) {
  LdsSym<NV> t;
#pragma unroll
  for (int v = 0; v < NV; v++) {
    t.v[2 * v] = x.l[v];
    t.v[2 * v + 1] = x.h[v];
  }
  row[lane] = t;
}

template <int NV>
__device__ __forceinline__ void lds_get(const LdsSym<NV> *row, uint32_t lane, Sym<NV> &x) {
  const LdsSym<NV> t = row[lane];
#pragma unroll
  for (int v = 0; v < NV; v++) {
    x.l[v] = t.v[2 * v];
    x.h[v] = t.v[2 * v + 1];
  }
}

// The scheduling barriers keep the compiler from hoisting the tables of many
// groups at once (each table is 21 SGPRs; hoisting spills SGPRs to VGPR lanes).
template <int NV>
__device__ __forceinline__ void ifft4(Sym<NV> &s0, Sym<NV> &s1, Sym<NV> &s2, Sym<NV> &s3, const RsTab *g) {
  __builtin_amdgcn_sched_barrier(0);
  const Tab m01 = dev::load_tab(g);
  dev::ifft_bf(s0, s1, m01);
  const Tab m23 = dev::load_tab(g + 2);
  dev::ifft_bf(s2, s3, m23);
  const Tab m02 = dev::load_tab(g + 1);
  dev::ifft_bf(s0, s2, m02);
  dev::ifft_bf(s1, s3, m02);
  __builtin_amdgcn_sched_barrier(0);
}

template <int NV>
__device__ __forceinline__ void fft4(Sym<NV> &s0, Sym<NV> &s1, Sym<NV> &s2, Sym<NV> &s3, const RsTab *g) {
  __builtin_amdgcn_sched_barrier(0);
  const Tab m02 = dev::load_tab(g + 1);
  dev::fft_bf(s0, s2, m02);
  dev::fft_bf(s1, s3, m02);
  const Tab m01 = dev::load_tab(g);
  dev::fft_bf(s0, s1, m01);
  const Tab m23 = dev::load_tab(g + 2);
  dev::fft_bf(s2, s3, m23);
  __builtin_amdgcn_sched_barrier(0);
}

// Four radix-4 groups that share one twiddle triple (stages d=4 and d=16 of a
// wave's layout): the three tables are loaded once for the four quads.
template <int NV>
__device__ __forceinline__ void ifft4x4(Sym<NV> *c, const RsTab *g) {
  __builtin_amdgcn_sched_barrier(0);
  const Tab m01 = dev::load_tab(g), m23 = dev::load_tab(g + 2), m02 = dev::load_tab(g + 1);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    dev::ifft_bf(c[i], c[i + 4], m01);
    dev::ifft_bf(c[i + 8], c[i + 12], m23);
    dev::ifft_bf(c[i], c[i + 8], m02);
    dev::ifft_bf(c[i + 4], c[i + 12], m02);
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <int NV>
__device__ __forceinline__ void fft4x4(Sym<NV> *c, const RsTab *g) {
  __builtin_amdgcn_sched_barrier(0);
  const Tab m02 = dev::load_tab(g + 1), m01 = dev::load_tab(g), m23 = dev::load_tab(g + 2);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    dev::fft_bf(c[i], c[i + 8], m02);
    dev::fft_bf(c[i + 4], c[i + 12], m02);
    dev::fft_bf(c[i], c[i + 4], m01);
    dev::fft_bf(c[i + 8], c[i + 12], m23);
  }
  __builtin_amdgcn_sched_barrier(0);
}

// ---- the same encode with each chunk's 63 twiddle tables staged in LDS and read
// back as VGPRs (broadcast ds_read_b128): no SGPR->VGPR moves for the v_perm
// operands and no SGPR spills (k_encode_ws64 holds 3 x 21-SGPR tables and spills
// ~120 SGPRs to VGPR lanes).
__device__ __forceinline__ Tab lds_tab(const uint4 *t) {  // one RsTab = 6 x uint4
  const uint4 q0 = t[0], q1 = t[1], q2 = t[2], q3 = t[3], q4 = t[4], q5 = t[5];
  Tab r;
  const uint32_t lo[10] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y};
  const uint32_t hi[10] = {q2.z, q2.w, q3.x, q3.y, q3.z, q3.w, q4.x, q4.y, q4.z, q4.w};
#pragma unroll
  for (int i = 0; i < 10; i++) {
    r.lo[i] = lo[i];
    r.hi[i] = hi[i];
  }
  r.flags = __builtin_amdgcn_readfirstlane(q5.x);  // uniform: scalar branch on XOR-only twiddles
  return r;
}

// group tables in plan order m01, m02, m23 (push_ifft_tabs / push_fft_tabs)
template <int NV>
__device__ __forceinline__ void ifft4l(Sym<NV> &s0, Sym<NV> &s1, Sym<NV> &s2, Sym<NV> &s3, const uint4 *g) {
  const Tab m01 = lds_tab(g), m02 = lds_tab(g + 6), m23 = lds_tab(g + 12);
  dev::ifft_bf(s0, s1, m01);
  dev::ifft_bf(s2, s3, m23);
  dev::ifft_bf(s0, s2, m02);
  dev::ifft_bf(s1, s3, m02);
}

template <int NV>
__device__ __forceinline__ void fft4l(Sym<NV> &s0, Sym<NV> &s1, Sym<NV> &s2, Sym<NV> &s3, const uint4 *g) {
  const Tab m01 = lds_tab(g), m02 = lds_tab(g + 6), m23 = lds_tab(g + 12);
  dev::fft_bf(s0, s2, m02);
  dev::fft_bf(s1, s3, m02);
  dev::fft_bf(s0, s1, m01);
  dev::fft_bf(s2, s3, m23);
}

template <int NV>
__global__ __launch_bounds__(kBlock) void k_encode_ws64l(EncodeArgs a) {
  constexpr int TI = 63;  // ifft_tab_count(64) == fft_tab_count(64)
  __shared__ LdsSym<NV> lds[64][64];
  __shared__ uint4 tl[TI * 6];
  const uint64_t sb = a.shard_bytes;
  const uint64_t regions = sb / 64 * (8 / NV) / 64;
  if (blockIdx.x >= regions) return;  // whole block: every wave shares the region
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t off = dev::lane_byte_offset<NV>(blockIdx.x, lane, a.contig);
  auto stage = [&](const RsTab *src) {
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
    for (uint32_t q = threadIdx.x; q < TI * 6; q += kBlock) tl[q] = s4[q];
  };
  const uint64_t s = blockIdx.y;
  const uint8_t *src = a.data + s * a.data_stripe_stride;
  Sym<NV> acc[16];
#pragma unroll
  for (int u = 0; u < 16; u++) dev::zero(acc[u]);
  for (uint32_t c = 0; c < a.n_chunks; c++) {
    const uint32_t t = c == 0 ? a.trunc_first : (c + 1 == a.n_chunks ? a.trunc_last : 64u);
    __syncthreads();  // previous chunk's readers of tl and lds are done
    stage(a.tabs + static_cast<uint64_t>(c) * TI);
    Sym<NV> cur[16];
#pragma unroll
    for (int j = 0; j < 16; j++) {  // layout A
      const uint32_t pos = 16 * w + j;
      if (pos < t && !skipped(a, c * 64 + pos))
        dev::load_sym_raw(cur[j], src + (static_cast<uint64_t>(c) * 64 + pos) * sb, off, a.contig);
      else dev::zero(cur[j]);
    }
#pragma unroll
    for (int j = 0; j < 16; j++) dev::pair_halves(cur[j], a.contig);
    __syncthreads();  // tables staged
#pragma unroll
    for (int g = 0; g < 4; g++) {  // stage d=1, groups r = 16w + 4g
      const uint32_t r = 16 * w + 4 * g;
      if (r < t) ifft4l(cur[4 * g], cur[4 * g + 1], cur[4 * g + 2], cur[4 * g + 3], tl + (r / 4 * 3) * 6);
    }
    if (16 * w < t) {  // stage d=4, group r = 16w
#pragma unroll
      for (int i = 0; i < 4; i++) ifft4l(cur[i], cur[i + 4], cur[i + 8], cur[i + 12], tl + (48 + w * 3) * 6);
    }
#pragma unroll
    for (int j = 0; j < 16; j++) lds_put(lds[16 * w + j], lane, cur[j]);
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 16; u++) lds_get(lds[(u & 3) + 4 * w + 16 * (u >> 2)], lane, cur[u]);  // layout B
#pragma unroll
    for (int i = 0; i < 4; i++) ifft4l(cur[i], cur[i + 4], cur[i + 8], cur[i + 12], tl + 60 * 6);  // d=16
#pragma unroll
    for (int u = 0; u < 16; u++) dev::xor_into(acc[u], cur[u]);  // root.zig:153-155
  }
  // FFT(0, 64, trunc m) on acc, root.zig:169
  __syncthreads();
  stage(a.tabs + static_cast<uint64_t>(a.n_chunks) * TI);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; i++) fft4l(acc[i], acc[i + 4], acc[i + 8], acc[i + 12], tl);  // d=16 (layout B)
#pragma unroll
  for (int u = 0; u < 16; u++) lds_put(lds[(u & 3) + 4 * w + 16 * (u >> 2)], lane, acc[u]);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 16; j++) lds_get(lds[16 * w + j], lane, acc[j]);  // layout A
  if (16 * w < a.m) {  // d=4, group r = 16w
#pragma unroll
    for (int i = 0; i < 4; i++) fft4l(acc[i], acc[i + 4], acc[i + 8], acc[i + 12], tl + (3 + w * 3) * 6);
  }
#pragma unroll
  for (int g = 0; g < 4; g++) {  // d=1, groups r = 16w + 4g
    const uint32_t r = 16 * w + 4 * g;
    if (r < a.m) fft4l(acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3], tl + (15 + r / 4 * 3) * 6);
  }
  uint8_t *dst = a.parity + s * a.parity_stripe_stride;
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const uint32_t pos = 16 * w + j;
    if (pos < a.m) dev::store_sym(dst + pos * sb, off, acc[j], a.contig);
  }
}

// ================================================= matrix reconstruct (e <= 8)
// restored_j = XOR_i M_ij(in_i): the reconstruct of root.zig:268-335 is
// GF(2)-linear in the received shards, so for one erasure pattern it is an
// n_out x n_in matrix of 16x16 GF(2) maps (host-derived, rs_plans.cpp). Each
// input is read once; its six bit-field selectors are shared by all n_out
// multiply-accumulates. Reads k shards, writes e: the algorithmic minimum.
template <int NV>
struct Sel {
  uint32_t a0[NV], a1[NV], a2[NV], b0[NV], b1[NV], b2[NV];
};

template <int NV>
__device__ __forceinline__ void make_sel(Sel<NV> &s, const Sym<NV> &y) {
#pragma unroll
  for (int v = 0; v < NV; v++) {
    s.a0[v] = y.l[v] & 0x07070707u;
    s.a1[v] = (y.l[v] >> 3) & 0x07070707u;
    s.a2[v] = (y.l[v] >> 6) & 0x03030303u;
    s.b0[v] = y.h[v] & 0x07070707u;
    s.b1[v] = (y.h[v] >> 3) & 0x07070707u;
    s.b2[v] = (y.h[v] >> 6) & 0x03030303u;
  }
}

template <int NV>
__device__ __forceinline__ void mac_sel(Sym<NV> &x, const Sel<NV> &s, const Tab &t) {
  using dev::perm;
  using dev::xor3;
#pragma unroll
  for (int v = 0; v < NV; v++) {
    uint32_t l = xor3(x.l[v], perm(t.lo[1], t.lo[0], s.a0[v]), perm(t.lo[3], t.lo[2], s.a1[v]));
    uint32_t h = xor3(x.h[v], perm(t.hi[1], t.hi[0], s.a0[v]), perm(t.hi[3], t.hi[2], s.a1[v]));
    l = xor3(l, perm(t.lo[4], t.lo[4], s.a2[v]), perm(t.lo[6], t.lo[5], s.b0[v]));
    h = xor3(h, perm(t.hi[4], t.hi[4], s.a2[v]), perm(t.hi[6], t.hi[5], s.b0[v]));
    x.l[v] = xor3(l, perm(t.lo[8], t.lo[7], s.b1[v]), perm(t.lo[9], t.lo[9], s.b2[v]));
    x.h[v] = xor3(h, perm(t.hi[8], t.hi[7], s.b1[v]), perm(t.hi[9], t.hi[9], s.b2[v]));
  }
}

// One received input of the matrix kernels: orig[idx] or rec[idx]; with
// kSrcXorScratch, rec[idx] ^ xs[idx] (a syndrome, reconstruct by syndromes).
// Split in two so a prefetched input keeps its loads in flight: issue_input only
// issues them, take_input waits, XORs the syndrome part and pairs the lane halves
// (the swap is a lane permutation, so it commutes with the XOR).
template <int NV>
struct InFlight {
  Sym<NV> y, z;
  bool x;
};

template <int NV>
__device__ __forceinline__ void issue_input(InFlight<NV> &f, int32_t src, const uint8_t *orig, const uint8_t *rec,
                                            const uint8_t *xs, uint64_t sb, uint32_t off, bool contig) {
  const uint64_t o = static_cast<uint64_t>(src & kSrcIndexMask) * sb;
  dev::load_sym_raw(f.y, ((src & kSrcRecovery) ? rec : orig) + o, off, contig);
  f.x = (src & kSrcXorScratch) != 0;
  if (f.x) dev::load_sym_raw(f.z, xs + o, off, contig);
}

template <int NV>
__device__ __forceinline__ void take_input(Sym<NV> &y, const InFlight<NV> &f, bool contig) {
  y = f.y;
  if (f.x) dev::xor_into(y, f.z);
  dev::pair_halves(y, contig);
}

template <int NV>
__device__ __forceinline__ void load_input(Sym<NV> &y, int32_t src, const uint8_t *orig, const uint8_t *rec,
                                           const uint8_t *xs, uint64_t sb, uint32_t off, bool contig) {
  InFlight<NV> f;
  issue_input(f, src, orig, rec, xs, sb, off, contig);
  take_input(y, f, contig);
}

template <int E, int NV, int D>
__global__ __launch_bounds__(kBlock) void k_decode_matrix(DecodeArgs a) {
  uint32_t off;
  if (!lane_offset<NV>(a.shard_bytes, a.contig, off)) return;
  const uint64_t sb = a.shard_bytes;
  typedef const __attribute__((address_space(4))) int32_t *CI;
  const uint32_t n_in = a.n_in;
  {  // one stripe per blockIdx.y (launches are split at 65535 stripes)
    const uint64_t s = blockIdx.y;
    const CI srcs = (CI)(a.pos_src + s * a.src_stride);
    const RsTab *mat = a.tab_mat + s * a.mat_stride;
    const uint32_t e_s = a.nout ? static_cast<uint32_t>(((CI)(a.nout))[s]) : static_cast<uint32_t>(E);
    const uint8_t *orig = a.orig + s * a.orig_stripe_stride;
    const uint8_t *rec = a.rec + s * a.rec_stripe_stride;
    const uint8_t *xs = a.xsrc + s * a.xsrc_stripe_stride;
    auto issue = [&](InFlight<NV> &f, uint32_t i) { issue_input(f, srcs[i], orig, rec, xs, sb, off, a.contig); };
    Sym<NV> acc[E];
#pragma unroll
    for (int j = 0; j < E; j++) dev::zero(acc[j]);
    if constexpr (D == 1) {
      // one input ahead: input i+1 in flight while input i is multiplied
      InFlight<NV> f;
      issue(f, 0);
      for (uint32_t i = 0; i < n_in; i++) {
        Sym<NV> y;
        take_input(y, f, a.contig);
        if (i + 1 < n_in) issue(f, i + 1);
        Sel<NV> sel;
        make_sel(sel, y);
        const RsTab *row = mat + static_cast<uint64_t>(i) * E;
#pragma unroll
        for (int j = 0; j < E; j++) mac_sel(acc[j], sel, dev::load_tab(row + j));
      }
    } else {
      // batches of D inputs: D loads in flight together, then D x E MACs
      for (uint32_t i0 = 0; i0 < n_in; i0 += D) {
        InFlight<NV> f[D];
#pragma unroll
        for (int d = 0; d < D; d++)
          if (i0 + d < n_in) issue(f[d], i0 + d);
#pragma unroll
        for (int d = 0; d < D; d++) {
          if (i0 + d >= n_in) break;
          Sym<NV> y;
          take_input(y, f[d], a.contig);
          Sel<NV> sel;
          make_sel(sel, y);
          const RsTab *row = mat + static_cast<uint64_t>(i0 + d) * E;
#pragma unroll
          for (int j = 0; j < E; j++) mac_sel(acc[j], sel, dev::load_tab(row + j));
        }
      }
    }
    uint8_t *out = a.out + s * a.out_stripe_stride;
#pragma unroll
    for (int j = 0; j < E; j++)
      if (static_cast<uint32_t>(j) < e_s) dev::store_sym(out + static_cast<uint64_t>(j) * sb, off, acc[j], a.contig);
  }
}

// ======================================= matrix reconstruct, output-tiled waves
// For 8 < e <= 64 (e.g. RS(200,55) losing all 55 data shards it can): a
// workgroup's 4 waves share the same 64 column units and split the e outputs,
// EW per wave ("per-wave output-shard tiling"); each wave streams all k inputs
// (the 4 waves read the same lines back to back: HBM once, L2 for the rest).
template <int NV>
__device__ __forceinline__ void mac_sel_v(Sym<NV> &x, const Sel<NV> &s, const uint32_t *lo, const uint32_t *hi) {
  using dev::perm;
  using dev::xor3;
#pragma unroll
  for (int v = 0; v < NV; v++) {
    uint32_t l = xor3(x.l[v], perm(lo[1], lo[0], s.a0[v]), perm(lo[3], lo[2], s.a1[v]));
    uint32_t h = xor3(x.h[v], perm(hi[1], hi[0], s.a0[v]), perm(hi[3], hi[2], s.a1[v]));
    l = xor3(l, perm(lo[4], lo[4], s.a2[v]), perm(lo[6], lo[5], s.b0[v]));
    h = xor3(h, perm(hi[4], hi[4], s.a2[v]), perm(hi[6], hi[5], s.b0[v]));
    x.l[v] = xor3(l, perm(lo[8], lo[7], s.b1[v]), perm(lo[9], lo[9], s.b2[v]));
    x.h[v] = xor3(h, perm(hi[8], hi[7], s.b1[v]), perm(hi[9], hi[9], s.b2[v]));
  }
}

// k_decode_mtile with the tables of each input row staged in LDS (double-buffered,
// one barrier per input) and read back as VGPRs by broadcast ds_read_b128; waves
// past n_out still stage and join the barriers, and padded outputs are skipped.
template <int EW, int NV>
__global__ __launch_bounds__(kBlock) void k_decode_mtile_lds(DecodeArgs a) {
  constexpr int kRow = 4 * EW;  // outputs per table row (4 waves)
  __shared__ uint4 tabs[2][kRow][5];  // lo[10] hi[10] of each RsTab
  const uint64_t sb = a.shard_bytes;
  if (blockIdx.x >= sb / 64 * (8 / NV) / 64) return;  // uniform over the block
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t j0 = w * EW;
  const uint32_t nj = j0 < a.n_out ? min(static_cast<uint32_t>(EW), a.n_out - j0) : 0u;
  const uint32_t off = dev::lane_byte_offset<NV>(blockIdx.x, lane, a.contig);
  const uint64_t s = blockIdx.y;
  typedef const __attribute__((address_space(4))) int32_t *CI;
  const CI srcs = (CI)(a.pos_src);
  const uint8_t *orig = a.orig + s * a.orig_stripe_stride;
  const uint8_t *rec = a.rec + s * a.rec_stripe_stride;
  const uint8_t *xs = a.xsrc + s * a.xsrc_stripe_stride;
  auto stage = [&](uint32_t i, int b) {
    const uint4 *src = reinterpret_cast<const uint4 *>(a.tab_mat + static_cast<uint64_t>(i) * kRow);
    for (uint32_t q = threadIdx.x; q < kRow * 5; q += kBlock) tabs[b][q / 5][q % 5] = src[q / 5 * 6 + q % 5];
  };
  Sym<NV> acc[EW];
#pragma unroll
  for (int j = 0; j < EW; j++) dev::zero(acc[j]);
  stage(0, 0);
  __syncthreads();
  InFlight<NV> f;
  if (nj) issue_input(f, srcs[0], orig, rec, xs, sb, off, a.contig);
  for (uint32_t i = 0; i < a.n_in; i++) {
    Sym<NV> y;
    if (nj) take_input(y, f, a.contig);
    if (i + 1 < a.n_in) {
      stage(i + 1, (i + 1) & 1);
      if (nj) issue_input(f, srcs[i + 1], orig, rec, xs, sb, off, a.contig);
    }
    if (nj) {
      Sel<NV> sel;
      make_sel(sel, y);
#pragma unroll
      for (int j = 0; j < EW; j++) {
        if (static_cast<uint32_t>(j) < nj) {  // uniform; keeps acc[] in registers (no dynamic index)
          const uint4 *t = tabs[i & 1][j0 + j];
          const uint4 q0 = t[0], q1 = t[1], q2 = t[2], q3 = t[3], q4 = t[4];
          const uint32_t lo[10] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y};
          const uint32_t hi[10] = {q2.z, q2.w, q3.x, q3.y, q3.z, q3.w, q4.x, q4.y, q4.z, q4.w};
          mac_sel_v(acc[j], sel, lo, hi);
        }
      }
    }
    __syncthreads();  // buffer (i & 1) free for input i + 2
  }
  uint8_t *out = a.out + s * a.out_stripe_stride;
#pragma unroll
  for (int j = 0; j < EW; j++)
    if (static_cast<uint32_t>(j) < nj) dev::store_sym(out + static_cast<uint64_t>(j0 + j) * sb, off, acc[j], a.contig);
}

// ============================================ generic: column walk in HBM scratch
template <int NV>
__device__ __forceinline__ void ld(Sym<NV> &s, const uint8_t *p) {
  typedef typename dev::VecT<NV>::type V;
  const V lo = *reinterpret_cast<const V *>(p), hi = *reinterpret_cast<const V *>(p + 32);
  if constexpr (NV == 1) {
    s.l[0] = lo;
    s.h[0] = hi;
  } else {
    for (int v = 0; v < NV; v++) {
      s.l[v] = lo[v];
      s.h[v] = hi[v];
    }
  }
}
template <int NV>
__device__ __forceinline__ void st(uint8_t *p, const Sym<NV> &s) {
  typedef typename dev::VecT<NV>::type V;
  V lo, hi;
  if constexpr (NV == 1) {
    lo = s.l[0];
    hi = s.h[0];
  } else {
    for (int v = 0; v < NV; v++) {
      lo[v] = s.l[v];
      hi[v] = s.h[v];
    }
  }
  *reinterpret_cast<V *>(p) = lo;
  *reinterpret_cast<V *>(p + 32) = hi;
}

// ---- the column transforms, phased (Generic.zig:15-147, runtime size / truncation).
// A layer-by-layer walk reads and writes the whole column once per layer (5 passes
// for 512 points). Here consecutive layers are grouped into phases whose butterflies
// close over n <= 64 positions pos0 + j*dlo (j < n): a phase loads such a set into
// VGPRs, runs its layers there (the j-space structure is exactly ifft_regs<n> /
// fft_regs<n>; twiddle groups and truncation use the real positions) and stores it
// back: 2 passes for 512 or 4,096 points. The first phase may read another buffer
// (positions >= n_src read as zero) and the last may write another (positions
// >= n_out dropped; out_sym: the shard layout of dev::store_sym), so a transform
// between buffers costs no copy pass.
struct XformIO {
  // buffers are wave-uniform bases; a lane adds `off` (global_load saddr + voffset form)
  const uint8_t *src;  // first phase input (positions >= n_src read as zero)
  uint64_t src_ps, n_src;
  uint8_t *work;       // intermediate phases (in place)
  uint64_t work_ps;
  uint8_t *out;        // last phase output (positions >= n_out not stored)
  uint64_t out_ps, n_out;
  bool out_sym, contig;  // out in the shard layout (dev::store_sym) instead of work's
  uint32_t off;          // the lane's byte offset in every buffer
};

template <int NV>
__device__ __forceinline__ void ldb(Sym<NV> &s, __amdgpu_buffer_rsrc_t r, uint32_t off) {
  static_assert(NV == 1, "generic column walk: one dword pair per lane");
  s.l[0] = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
  s.h[0] = __builtin_amdgcn_raw_buffer_load_b32(r, off + 32u, 0, 0);
}
template <int NV>
__device__ __forceinline__ void stb(__amdgpu_buffer_rsrc_t r, uint32_t off, const Sym<NV> &s) {
  __builtin_amdgcn_raw_buffer_store_b32(s.l[0], r, off, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b32(s.h[0], r, off + 32u, 0, 0);
}

template <int N, int NV, bool INV>
__device__ __forceinline__ void xform_phase(const XformIO &io, bool first, bool last, const RsTab *__restrict__ tabs,
                                         uint64_t ti, uint64_t size, uint64_t rmax, uint32_t dlo_log) {
  const uint8_t *src = first ? io.src : io.work;
  const uint64_t sps = first ? io.src_ps : io.work_ps, n_src = first ? io.n_src : size;
  uint8_t *dst = last ? io.out : io.work;
  const uint64_t dps = last ? io.out_ps : io.work_ps, n_dst = last ? io.n_out : size;
  const bool sym = last && io.out_sym;
  const uint64_t dlo = 1ull << dlo_log, span = static_cast<uint64_t>(N) << dlo_log;
  for (uint64_t blk = 0; blk < size; blk += span) {
    if (!INV && blk >= n_dst) break;  // FFT: a block past the stored outputs feeds nothing later
    for (uint64_t lo = 0; lo < dlo; lo++) {
      // opaque per sub-problem: the N row offsets (j << dlo_log) * ps and the group tables are
      // computed where used instead of hoisted out of the walk and spilled (see opq)
      const uint32_t dl = opqu(dlo_log);
      const RsTab *tb = opq(tabs);
      Sym<NV> s[N];
#pragma unroll
      for (int j = 0; j < N; j++) {
        const uint64_t p = blk + lo + (static_cast<uint64_t>(j) << dl);
        if (p < n_src) ldb(s[j], row_rsrc(src + p * sps), io.off);
        else dev::zero(s[j]);
      }
      if constexpr (INV) ifft_sub<N, NV>(s, tb, ti, size, rmax, blk, dl);
      else fft_sub<N, NV>(s, tb, ti, size, rmax, blk, dl);
#pragma unroll
      for (int j = 0; j < N; j++) {
        const uint64_t p = blk + lo + (static_cast<uint64_t>(j) << dl);
        if (p < n_dst) {
          if (sym) dev::store_sym(dst + p * dps, io.off, s[j], io.contig);
          else stb(row_rsrc(dst + p * dps), io.off, s[j]);
        }
      }
    }
  }
}

// the whole transform of `size` points (a power of two) with truncation `trunc`
template <int NV, bool INV>
__device__ __forceinline__ void xform_ph(const XformIO &io, uint64_t size, uint64_t trunc, const RsTab *__restrict__ tabs) {
  const uint32_t lg = log2_u64(size), n4 = lg / 2;
  const bool r2 = lg & 1;
  const uint64_t rmax = trunc < size ? trunc : size;
  uint64_t ti = 0;
  uint32_t layer = 0;  // radix-4 layers done (IFFT: from distance 1 up; FFT: from size/4 down)
  bool r2_done = !r2, first = true;
  do {
    const uint32_t c = n4 - layer < 3 ? n4 - layer : 3;
    const bool with_r2 = !r2_done && layer + c == n4 && c < 3;
    const uint32_t n = (1u << (2 * c)) << (with_r2 ? 1 : 0);
    const bool last = layer + c == n4 && (r2_done || with_r2);
    // lowest distance of the phase (its position stride)
    const uint32_t dlo_log = INV ? 2 * layer : (with_r2 || c == 0 ? 0 : lg - 2 * (layer + c));
#define RS_XF_CASE(N_) \
  case N_: xform_phase<N_, NV, INV>(io, first, last, tabs, ti, size, rmax, dlo_log); break;
    switch (n) {
      RS_XF_CASE(1) RS_XF_CASE(2) RS_XF_CASE(4) RS_XF_CASE(8) RS_XF_CASE(16) RS_XF_CASE(32) RS_XF_CASE(64)
    }
#undef RS_XF_CASE
    for (uint32_t l = layer; l < layer + c; l++) ti += INV ? 3 * (size >> (2 * l + 2)) : 3ull << (2 * l);
    layer += c;
    r2_done = r2_done || with_r2;
    first = false;
    if (c == 0) r2_done = true;  // the lone radix-2 phase (n == 2) just ran
  } while (layer < n4 || !r2_done);
}

// in place on positions w + p*ps + off (the former layer-by-layer ifft_mem / fft_mem)
template <int NV>
__device__ __forceinline__ void ifft_mem(uint8_t *w, uint32_t off, uint64_t ps, uint64_t size, uint64_t trunc,
                         const RsTab *__restrict__ tabs) {
  const XformIO io{w, ps, size, w, ps, w, ps, size, false, false, off};
  xform_ph<NV, true>(io, size, trunc, tabs);
}
template <int NV>
__device__ __forceinline__ void fft_mem(uint8_t *w, uint32_t off, uint64_t ps, uint64_t size, uint64_t trunc,
                        const RsTab *__restrict__ tabs) {
  const XformIO io{w, ps, size, w, ps, w, ps, size, false, false, off};
  xform_ph<NV, false>(io, size, trunc, tabs);
}

template <int NV>
__device__ __forceinline__ void xor_mem(uint8_t *a, const uint8_t *b) {
  Sym<NV> x, y;
  ld(x, a);
  ld(y, b);
  dev::xor_into(x, y);
  st(a, x);
}

template <int NV>
__global__ __launch_bounds__(kBlock) void k_encode_generic(EncodeArgs a) {
  uint32_t off;
  if (!lane_offset<NV>(a.shard_bytes, a.contig, off)) return;
  const uint64_t sb = a.shard_bytes, C = a.chunk;
  for (uint64_t s = blockIdx.y; s < a.n_stripes; s += gridDim.y) {
    const uint8_t *src = a.data + s * a.data_stripe_stride + off;
    uint8_t *work = a.scratch + s * a.work * sb + off;
    for (uint32_t j = 0; j < a.n_chunks; j++) {
      const uint64_t t = j == 0 ? a.trunc_first : (j + 1 == a.n_chunks ? a.trunc_last : C);
      for (uint64_t p = 0; p < C; p++) {
        Sym<NV> v;
        if (p < t && !skipped(a, static_cast<uint32_t>(j * C + p))) ld(v, src + (j * C + p) * sb);
        else dev::zero(v);
        st(work + (j * C + p) * sb, v);
      }
      ifft_mem<NV>(work - off + j * C * sb, off, sb, C, t, a.tabs + static_cast<uint64_t>(j) * a.tabs_per_chunk);
      if (j > 0)
        for (uint64_t p = 0; p < C; p++) xor_mem<NV>(work + p * sb, work + (j * C + p) * sb);
    }
    fft_mem<NV>(work - off, off, sb, C, a.m, a.tabs + static_cast<uint64_t>(a.n_chunks) * a.tabs_per_chunk);
    uint8_t *dst = a.parity + s * a.parity_stripe_stride + off;
    for (uint64_t p = 0; p < a.m; p++) {
      Sym<NV> v;
      ld(v, work + p * sb);
      dev::store_sym(dst + p * sb, 0u, v, a.contig);
    }
  }
}

// Formal derivative (root.zig:306-312): for i in [1, W), w[i - lowbit(i) + j] ^= w[i + j]
// for j < lowbit(i). Reads lie at or above i and writes below it, so every read sees an
// original value: out[p] = in[p] ^ XOR over clear bits b of p (b < log2 W) of in[p + 2^b]
// (k_dec_deriv: 64-position blocks, the low 6 bits combined in VGPRs in ascending order,
// the high bits as partner blocks; one independent load per term).

// ---- the generic reconstruct as a launch sequence (launch_decode_generic): one launch per
// phase of xform_ph, the phase's sub-problems across the grid (y), so a small batch still
// fills the chip. Grid: x = column units, y = sub-problem, z = stripes (strided).
// Per stripe the scratch holds X (W positions: the IFFT, in place; then A, written over X by
// the first FFT phase) and B (the positions the truncated FFT still needs after its first
// phase; decode_generic_rows). The steps ride
// on the phases:
//  * GATHER (first IFFT phase): positions come from the received shards * pre, zero where
//    nothing was received (root.zig:291-303), instead of a staging pass;
//  * the IFFT writes only positions < round_up(trunc, span): a sub-problem past the
//    truncation is all zero and so is what it would write (the next phase reads zeros);
//  * the formal derivative (root.zig:306-312) is out[p] = in[p] ^ XOR over clear bits b of
//    p of in[p + 2^b] (every read an original value): D = I + H + L, H the bits the first
//    FFT phase F1 holds (it spans every position), L the bits below its stride. L acts on
//    the low bits only and F1 on the high bits only (its twiddles depend on the group, not
//    on the low bits), so F1 D = F1 (I + H) + L F1. DERIV (first FFT phase): H in VGPRs
//    (ascending, reads above writes), A = F1((I + H) X); SPLITB: the same sub-problem
//    again without H, B = F1(X); LSUM (second FFT phase): A + L B, L's bits the
//    sub-problem holds in VGPRs, the ones below its stride as loads of B (none for
//    W = 2048). No partner loads of X (tests/test_decode_phases_model.py checks this
//    against the layer-by-layer decode);
//  * the FFT writes only positions < round_up(trunc_fft, span) and skips sub-problems past
//    the truncation (their outputs feed nothing: root.zig:318 reads [0, trunc));
//  * SCATTER (last FFT phase): only the erased positions, * post, into the restored rows
//    (root.zig:320-326).
enum : int { kPhGather = 1, kPhDeriv = 2, kPhScatter = 4, kPhSplitB = 8, kPhLsum = 16 };

struct PhaseArgs {
  const uint8_t *src;  // stripe s's input: src + s * src_stride, position p at + p * sb
  uint8_t *dst;        // output (in place: dst == src)
  uint64_t src_stride, dst_stride, n_src, n_dst;  // positions >= n_src read as zero, >= n_dst not stored
  uint64_t sb, size, rmax, ti;
  const RsTab *tabs;
  uint32_t dlo_log;
  const uint8_t *src2;  // LSUM: B (stride src_stride)
  uint8_t *dst2;        // SPLITB: B (stride dst_stride)
  bool contig;          // shard rows in the contiguous lane layout (shard_bytes % 512 == 0)
  // NI > 0 (the first FFT phase): the IFFT's last phase runs on the loaded rows first
  const RsTab *tabs_i;
  uint64_t ti_i, rmax_i;
  uint32_t dlo_i;
  // k_ephase SYN (low-rate block form): the recovery rows and the syndrome multipliers
  const uint8_t *rec = nullptr;
  uint64_t rec_stride = 0;
  const int32_t *syn_idx = nullptr;
  const RsTab *syn_tab = nullptr;
};

// Table pointers made opaque inside the stripe / pass loops: a group's table loads are then
// issued where the group runs. Hoisted out of the loops (the tables do not depend on the
// stripe), every group's tables stayed live across them, 21 SGPRs each: 1,200-2,300 SGPRs
// spilled into VGPR lanes per 64-point phase kernel and 250+ VGPRs, one wave per SIMD (round 5).
__device__ __forceinline__ PhaseArgs opq(const PhaseArgs &q) {
  PhaseArgs r = q;
  r.tabs = opq(r.tabs);
  r.tabs_i = opq(r.tabs_i);
  r.syn_tab = opq(r.syn_tab);
  r.dlo_log = opqu(r.dlo_log);  // the row offsets (blk + lo + (j << dlo_log)) * sb likewise
  return r;
}

// The IFFT's last phase inside the first FFT phase's sub-problem: that sub-problem (fixed
// position bits below dlo_f, registers j over the bits above) is the union of G = N / NI of
// the IFFT phase's sub-problems (bits below dlo_i = dlo_f + log2 G fixed): group g holds
// registers g + t G, t < NI (tests/test_decode_phases_model.py)
template <int N, int NI>
__device__ __forceinline__ void ifft_last_in(Sym<1> *v, const PhaseArgs &q) {
  if constexpr (NI > 0) {
    constexpr int G = N / NI;
#pragma unroll
    for (int g = 0; g < G; g++) {
      Sym<1> w[NI];
#pragma unroll
      for (int t = 0; t < NI; t++) w[t] = v[g + t * G];
      ifft_sub<NI, 1>(w, opq(q.tabs_i), q.ti_i, q.size, q.rmax_i, 0, q.dlo_i);  // the groups share tables
#pragma unroll
      for (int t = 0; t < NI; t++) v[g + t * G] = w[t];
    }
  }
}

// scratch rows (X, A, B): lane u's 4 symbols as one 8-byte (lo, hi) pair at u * 8, so a
// wave's access is 512 contiguous bytes (one dwordx2 per lane); only the shard rows keep the
// reference's chunk layout (Generic.zig:152-156)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void ldp(Sym<1> &s, __amdgpu_buffer_rsrc_t r, uint32_t o) {
  const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, o, 0, 0);
  s.l[0] = v.x;
  s.h[0] = v.y;
}
__device__ __forceinline__ void stp(__amdgpu_buffer_rsrc_t r, uint32_t o, const Sym<1> &s) {
  u32x2 v;
  v.x = s.l[0];
  v.y = s.h[0];
  __builtin_amdgcn_raw_buffer_store_b64(v, r, o, 0, 0);
}

template <int N, bool INV, int MODE, int NI = 0>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3))) void k_dphase(DecodeArgs a, PhaseArgs q0) {
  const PhaseArgs &q = q0;
  // lane unit u (4 symbols of one shard column); lanes past the shard's last unit stay (the
  // lane reads below need every lane): they load at offset 0 and store nothing
  const uint64_t sb = q.sb, u = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  const bool act = u < sb / 8;
  const uint32_t so = act ? static_cast<uint32_t>(u * 8) : 0u;  // scratch offset
  // shard-row offset: the contiguous lane layout (512-B waves, lo / hi halves paired by a
  // lane swap) where the shard is whole 512-B waves, else 4 + 4 bytes of one 64-B chunk
  const uint32_t io = act ? dev::lane_byte_offset<1>(u / 64, static_cast<uint32_t>(u % 64), q.contig) : 0u;
  const uint32_t io_h = io + (q.contig ? 256u : 32u);
  const uint64_t sub = blockIdx.y, dlo = 1ull << q.dlo_log;
  const uint64_t blk = (sub >> q.dlo_log) * (static_cast<uint64_t>(N) << q.dlo_log), lo = sub & (dlo - 1);
  for (uint64_t s = blockIdx.z; s < a.n_stripes; s += gridDim.z) {
    const PhaseArgs q = opq(q0);
    Sym<1> v[N];
    if constexpr ((MODE & kPhSplitB) != 0) {  // B = F1(X), the sub-problem without H: first,
      // since A is then written over X (in place: the lane reads its positions before it
      // writes them, and no other lane or workgroup touches them; decode_generic_rows)
      const uint8_t *x = q.src + s * q.src_stride;
      uint8_t *y = q.dst2 + s * q.dst_stride;
#pragma unroll
      for (int j = 0; j < N; j++) {
        const uint64_t p = blk + lo + (static_cast<uint64_t>(j) << q.dlo_log);
        if (p < q.n_src) ldp(v[j], row_rsrc(x + p * sb), so);
        else dev::zero(v[j]);
      }
      ifft_last_in<N, NI>(v, q);
      fft_sub<N, 1>(v, q.tabs, q.ti, q.size, q.rmax, blk, q.dlo_log);
      const uint32_t dls = opqu(q.dlo_log);  // store offsets recomputed, not held across the transform
#pragma unroll
      for (int j = 0; j < N; j++) {
        const uint64_t p = blk + lo + (static_cast<uint64_t>(j) << dls);
        if (act && p < q.n_dst) stp(row_rsrc(y + p * sb), so, v[j]);
      }
    }
    if constexpr ((MODE & kPhGather) != 0) {
      // the sub-problem's sources in one vector load (lane j: position j), then per position
      // a lane read and a load through a buffer resource with no records when nothing was
      // received (reads zero): no scalar load, wait and branch in front of every load
      const uint8_t *orig = a.orig + s * a.orig_stripe_stride;
      const uint8_t *rec = a.rec + s * a.rec_stripe_stride;
      const RsTab *tab_pre = a.tab_pre + s * a.pattern_stride;
      const int32_t *pos_src = a.pos_src + s * a.pattern_stride;
      const uint32_t ln = __lane_id();
      const uint64_t lp = blk + lo + (static_cast<uint64_t>(ln) << q.dlo_log);
      const int32_t my = ln < static_cast<uint32_t>(N) && lp < q.n_src ? pos_src[lp] : -1;
      int32_t srcs[N];
#pragma unroll
      for (int j = 0; j < N; j++) {
        srcs[j] = __builtin_amdgcn_readlane(my, j);
        const uint8_t *row = ((srcs[j] & kSrcRecovery) ? rec : orig) + static_cast<uint64_t>(srcs[j] & kSrcIndexMask) * sb;
        const __amdgpu_buffer_rsrc_t r = srcs[j] >= 0 ? row_rsrc(row) : zero_rsrc();
        v[j].l[0] = __builtin_amdgcn_raw_buffer_load_b32(r, io, 0, 0);
        v[j].h[0] = __builtin_amdgcn_raw_buffer_load_b32(r, io_h, 0, 0);
      }
      if (q.contig)  // pair after every load is issued (a swap behind its own load waits for it)
#pragma unroll
        for (int j = 0; j < N; j++) dev::pair_halves(v[j], true);
#pragma unroll
      for (int j = 0; j < N; j++) {
        if (srcs[j] >= 0) dev::mul_inplace(v[j], dev::load_tab(tab_pre + blk + lo + (static_cast<uint64_t>(j) << q.dlo_log)));
        group_fence();
      }
    } else if constexpr ((MODE & kPhLsum) != 0) {
      const uint8_t *A = q.src + s * q.src_stride, *B = q.src2 + s * q.src_stride;
#pragma unroll
      for (int j = 0; j < N; j++) {
        const uint64_t p = blk + lo + (static_cast<uint64_t>(j) << q.dlo_log);
        if (p < q.n_src) ldp(v[j], row_rsrc(B + p * sb), so);
        else dev::zero(v[j]);
      }
#pragma unroll
      for (int j = 0; j < N; j++) {  // L's bits in VGPRs: v[j] = XOR over clear bits of B[j + bb]
        Sym<1> t;
        dev::zero(t);
#pragma unroll
        for (int bb = 1; bb < N; bb <<= 1)
          if (!(j & bb)) dev::xor_into(t, v[j + bb]);
        v[j] = t;
      }
      for (uint32_t b = 0; b < q.dlo_log; b++) {  // L's bits below the stride: loads of B
        if ((lo >> b) & 1) continue;                // wave-uniform
#pragma unroll
        for (int j = 0; j < N; j++) {
          const uint64_t p = blk + lo + (1ull << b) + (static_cast<uint64_t>(j) << q.dlo_log);
          if (p < q.n_src) {
            Sym<1> t;
            ldp(t, row_rsrc(B + p * sb), so);
            dev::xor_into(v[j], t);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < N; j++) {
        const uint64_t p = blk + lo + (static_cast<uint64_t>(j) << q.dlo_log);
        if (p < q.n_src) {
          Sym<1> t;
          ldp(t, row_rsrc(A + p * sb), so);
          dev::xor_into(v[j], t);
        }
      }
    } else {
      const uint8_t *x = q.src + s * q.src_stride;
      const uint32_t dll = opqu(q.dlo_log);  // not the SPLITB loads' offsets, held across its FFT
#pragma unroll
      for (int j = 0; j < N; j++) {
        const uint64_t p = blk + lo + (static_cast<uint64_t>(j) << dll);
        if (p < q.n_src) ldp(v[j], row_rsrc(x + p * sb), so);
        else dev::zero(v[j]);
      }
      ifft_last_in<N, NI>(v, q);
      if constexpr ((MODE & kPhDeriv) != 0) {  // H: the bits this sub-problem holds
#pragma unroll
        for (int j = 0; j < N; j++)
#pragma unroll
          for (int bb = 1; bb < N; bb <<= 1)
            if (!(j & bb)) dev::xor_into(v[j], v[j + bb]);
      }
    }
    if constexpr (INV) ifft_sub<N, 1>(v, q.tabs, q.ti, q.size, q.rmax, blk, q.dlo_log);
    else fft_sub<N, 1>(v, q.tabs, q.ti, q.size, q.rmax, blk, q.dlo_log);
    if constexpr ((MODE & kPhScatter) != 0) {
      uint8_t *out = a.out + s * a.out_stripe_stride;
      const RsTab *tab_post = a.tab_post + s * a.pattern_stride;
      const int32_t *pos_dst = a.pos_dst + s * a.pattern_stride;
      const uint32_t ln = __lane_id();
      const uint64_t lp = blk + lo + (static_cast<uint64_t>(ln) << q.dlo_log);
      const int32_t my = ln < static_cast<uint32_t>(N) && lp < q.rmax ? pos_dst[lp] : -1;
#pragma unroll
      for (int j = 0; j < N; j++) {
        const int32_t dst = __builtin_amdgcn_readlane(my, j);
        if (dst >= 0) {  // wave-uniform
          dev::mul_inplace(v[j], dev::load_tab(tab_post + blk + lo + (static_cast<uint64_t>(j) << q.dlo_log)));
          if (q.contig) dev::pair_halves(v[j], true);  // back to the lo / hi halves (an involution)
          const __amdgpu_buffer_rsrc_t r = act ? row_rsrc(out + static_cast<uint64_t>(dst) * sb) : zero_rsrc();
          __builtin_amdgcn_raw_buffer_store_b32(v[j].l[0], r, io, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(v[j].h[0], r, io_h, 0, 0);
        }
        group_fence();
      }
    } else {
      uint8_t *y = q.dst + s * q.dst_stride;
      const uint32_t dls = opqu(q.dlo_log);  // store offsets recomputed, not held across the transform
#pragma unroll
      for (int j = 0; j < N; j++) {
        const uint64_t p = blk + lo + (static_cast<uint64_t>(j) << dls);
        if (act && p < q.n_dst) stp(row_rsrc(y + p * sb), so, v[j]);
      }
    }
  }
}

// ---- the low-rate generic encode as one launch per transform phase (launch_encode_low_phases):
// coefficients = IFFT_C(originals at [0, k), trunc k) in region 0 of the stripe's scratch
// (the first phase gathers the original rows); recovery chunk j = FFT_C(coefficients, skew
// (j+1)C, trunc t_j = min(C, m - jC)) in region 1 + (j - chunk0), its last phase storing
// the recovery rows jC + p directly. The IFFT's last phase runs inside the first FFT
// phase's loads (as launch_decode_generic does), so region 0 is read, never rewritten, by
// every chunk. Grid y = (chunk of the launch, sub-problem) for the FFT phases.
// SYN (the low-rate reconstruct in block form, launch_low_blocks): the last FFT phase of block
// K = j + 1 forms the residual's syndromes instead of storing recovery rows, and the gather
// reads the originals flagged in a.skip (the erased ones) as zero.
// DLO (an IFFT phase of 64 contiguous positions, launch_low_blocks): besides its output U, the
// phase stores W = ((1 + gamma) I + D_lo) U to dst2 (1 + gamma: the block's table at syn_tab),
// D_lo the formal derivative's terms over the bits the phase holds (bits 0-5): the later IFFT
// phases act on higher bits with twiddles that do not depend on these, so they commute with D_lo
// and k_lbfin1 gets (1 + gamma) U + D_lo U of the final IFFT output by running the last IFFT
// phase on W.
enum : int { kEpGather = 1, kEpOut = 2, kEpFft = 4, kEpSyn = 8, kEpDlo = 16 };

template <int N, int MODE, int NI>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3))) void k_ephase(EncodeArgs a, PhaseArgs q0, uint32_t subs, uint32_t from_chunk) {
  const PhaseArgs &q = q0;
  const uint64_t sb = q.sb, u = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  const bool act = u < sb / 8;
  const uint32_t so = act ? static_cast<uint32_t>(u * 8) : 0u;
  const uint32_t io = act ? dev::lane_byte_offset<1>(u / 64, static_cast<uint32_t>(u % 64), q.contig) : 0u;
  const uint32_t io_h = io + (q.contig ? 256u : 32u);
  constexpr bool kFft = (MODE & kEpFft) != 0;
  const uint64_t C = q.size, dlo = 1ull << q.dlo_log;
  const uint32_t sl = static_cast<uint32_t>(__builtin_ctz(subs | (1u << 31)));  // subs: a power of two
  const uint32_t ch = kFft ? blockIdx.y >> sl : 0u;  // chunk of this launch (scalar shifts, not a VALU divide)
  const uint64_t sub = kFft ? blockIdx.y & (subs - 1) : blockIdx.y;
  const uint64_t blk = (sub >> q.dlo_log) * (static_cast<uint64_t>(N) << q.dlo_log), lo = sub & (dlo - 1);
  const uint64_t j = a.chunk0 + ch;  // recovery chunk
  const uint64_t rmax = kFft ? (a.m - j * C < C ? a.m - j * C : C) : q.rmax;
  if (kFft && blk >= rmax) return;  // wave-uniform: outputs past the chunk's truncation feed nothing
  const uint64_t n_dst = kFft ? (rmax + dlo - 1) / dlo * dlo : q.n_dst;  // what later phases read
  for (uint64_t s = blockIdx.z; s < a.n_stripes; s += gridDim.z) {
    const PhaseArgs q = opq(q0);
    const RsTab *tabs = kFft ? q.tabs + j * a.tabs_per_chunk : q.tabs;
    Sym<1> v[N];
    const uint8_t *x = q.src + s * q.src_stride + (from_chunk ? (1 + ch) * C * sb : 0);
    if constexpr ((MODE & kEpGather) != 0) {
      const uint8_t *d = a.data + s * a.data_stripe_stride;
#pragma unroll
      for (int jj = 0; jj < N; jj++) {
        const uint64_t p = blk + lo + (static_cast<uint64_t>(jj) << q.dlo_log);
        const bool rd = p < q.n_src && !skipped(a, static_cast<uint32_t>(p));
        const __amdgpu_buffer_rsrc_t r = rd ? row_rsrc(d + p * sb) : zero_rsrc();
        v[jj].l[0] = __builtin_amdgcn_raw_buffer_load_b32(r, io, 0, 0);
        v[jj].h[0] = __builtin_amdgcn_raw_buffer_load_b32(r, io_h, 0, 0);
      }
      if (q.contig)
#pragma unroll
        for (int jj = 0; jj < N; jj++) dev::pair_halves(v[jj], true);
    } else {
#pragma unroll
      for (int jj = 0; jj < N; jj++) {
        const uint64_t p = blk + lo + (static_cast<uint64_t>(jj) << q.dlo_log);
        if (p < q.n_src) ldp(v[jj], row_rsrc(x + p * sb), so);
        else dev::zero(v[jj]);
      }
      ifft_last_in<N, NI>(v, q);
    }
    if constexpr (kFft) fft_sub<N, 1>(v, tabs, q.ti, C, rmax, blk, q.dlo_log);
    else ifft_sub<N, 1>(v, tabs, q.ti, C, rmax, blk, q.dlo_log);
    if constexpr ((MODE & kEpSyn) != 0) {
      // recovery row r = jC + p: (rec_r ^ Enc(d')_r) L_r sigma_K where r is a row used, else
      // zero; the rows in groups of 8 loads (lane jj holds position jj's row flag)
      const uint8_t *rc = q.rec + s * q.rec_stride + j * C * sb;
      const int32_t *si = q.syn_idx + j * C;
      const RsTab *st = q.syn_tab + j * C;
      uint8_t *y = q.dst + s * q.dst_stride + (1 + ch) * C * sb;
      const uint32_t ln = __lane_id();
      const uint64_t lp = blk + lo + (static_cast<uint64_t>(ln) << q.dlo_log);
      const int32_t my = ln < static_cast<uint32_t>(N) && lp < rmax ? si[lp] : -1;
      constexpr int G8 = N < 8 ? N : 8;
#pragma unroll
      for (int g0 = 0; g0 < N; g0 += G8) {
        Sym<1> t[G8];
#pragma unroll
        for (int jj = 0; jj < G8; jj++) {
          const uint64_t p = blk + lo + (static_cast<uint64_t>(g0 + jj) << q.dlo_log);
          const bool used = __builtin_amdgcn_readlane(my, g0 + jj) >= 0;
          const __amdgpu_buffer_rsrc_t r = used ? row_rsrc(rc + p * sb) : zero_rsrc();  // wave-uniform
          t[jj].l[0] = __builtin_amdgcn_raw_buffer_load_b32(r, io, 0, 0);
          t[jj].h[0] = __builtin_amdgcn_raw_buffer_load_b32(r, io_h, 0, 0);
        }
        if (q.contig)
#pragma unroll
          for (int jj = 0; jj < G8; jj++) dev::pair_halves(t[jj], true);
#pragma unroll
        for (int jj = 0; jj < G8; jj++) {
          const uint64_t p = blk + lo + (static_cast<uint64_t>(g0 + jj) << q.dlo_log);
          if (__builtin_amdgcn_readlane(my, g0 + jj) >= 0) {  // wave-uniform
            dev::xor_into(v[g0 + jj], t[jj]);
            dev::mul_inplace(v[g0 + jj], dev::load_tab(st + p));
          } else {
            dev::zero(v[g0 + jj]);
          }
          if (act && p < rmax) stp(row_rsrc(y + p * sb), so, v[g0 + jj]);
          group_fence();
        }
      }
    } else if constexpr ((MODE & kEpOut) != 0) {
      uint8_t *par = a.parity + s * a.parity_stripe_stride + j * C * sb;
#pragma unroll
      for (int jj = 0; jj < N; jj++) {
        const uint64_t p = blk + lo + (static_cast<uint64_t>(jj) << q.dlo_log);
        if (p < rmax) {  // wave-uniform
          if (q.contig) dev::pair_halves(v[jj], true);
          const __amdgpu_buffer_rsrc_t r = act ? row_rsrc(par + p * sb) : zero_rsrc();
          __builtin_amdgcn_raw_buffer_store_b32(v[jj].l[0], r, io, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(v[jj].h[0], r, io_h, 0, 0);
        }
      }
    } else {
      uint8_t *y = q.dst + s * q.dst_stride + (kFft ? (1 + ch) * C * sb : 0);
      const uint32_t dls = opqu(q.dlo_log);  // store offsets recomputed, not held across the transform
#pragma unroll
      for (int jj = 0; jj < N; jj++) {
        const uint64_t p = blk + lo + (static_cast<uint64_t>(jj) << dls);
        if (act && p < n_dst) stp(row_rsrc(y + p * sb), so, v[jj]);
      }
      if constexpr ((MODE & kEpDlo) != 0) {  // W = ((1 + gamma) I + D_lo) U, ascending (reads above writes)
        const Tab g1 = dev::load_tab(q.syn_tab);
#pragma unroll
        for (int jj = 0; jj < N; jj++) {
          Sym<1> t = v[jj];
          dev::mul_inplace(t, g1);
#pragma unroll
          for (int bb = 1; bb < N; bb <<= 1)
            if (!(jj & bb)) dev::xor_into(t, v[jj + bb]);
          v[jj] = t;
          group_fence();
        }
        uint8_t *w = q.dst2 + s * q.dst_stride;
        const uint32_t dlw = opqu(q.dlo_log);
#pragma unroll
        for (int jj = 0; jj < N; jj++) {
          const uint64_t p = blk + lo + (static_cast<uint64_t>(jj) << dlw);
          if (act && p < n_dst) stp(row_rsrc(w + p * sb), so, v[jj]);
        }
      }
    }
  }
}

// The final FFT's first phase for the block form with the derivative applied whole before it
// (IFFTs of two phases, C <= 4096): block K's U = IFFT_last(U_pre) and
// IFFT_last(W) = (1 + gamma) U + D_lo U (W from k_ephase DLO) are formed in VGPRs, then
// Z = D_hi U + IFFT_last(W) = D_C U + gamma U (D_hi: the derivative's terms over the bits the
// last IFFT phase holds, register bits >= G = N / NI of this sub-problem) for u = 1, Z = U for
// u = 0, and A' += F1(Z) (acc: add to what an earlier block stored). The next phase is then a
// plain FFT phase with the scatter: no B' and no LSUM.
template <int NI>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3))) void k_lbfin1(uint64_t n_stripes,
                                                                                         PhaseArgs q0, uint32_t u,
                                                                                         uint32_t acc) {
  const PhaseArgs &q = q0;
  constexpr int N = 64, G = N / NI;
  const uint64_t sb = q.sb, uu = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  const bool act = uu < sb / 8;
  const uint32_t so = act ? static_cast<uint32_t>(uu * 8) : 0u;
  const uint64_t sub = blockIdx.y, dlo = 1ull << q.dlo_log;
  const uint64_t blk = (sub >> q.dlo_log) * (static_cast<uint64_t>(N) << q.dlo_log), lo = sub & (dlo - 1);
  for (uint64_t s = blockIdx.z; s < n_stripes; s += gridDim.z) {
    const PhaseArgs q = opq(q0);
    const uint8_t *x = q.src + s * q.src_stride;
    Sym<1> v[N];
#pragma unroll
    for (int j = 0; j < N; j++) {
      const uint64_t p = blk + lo + (static_cast<uint64_t>(j) << q.dlo_log);
      if (p < q.n_src) ldp(v[j], row_rsrc(x + p * sb), so);
      else dev::zero(v[j]);
    }
    ifft_last_in<N, NI>(v, q);
    if (u) {
#pragma unroll
      for (int j = 0; j < N; j++) {  // D_hi U, ascending (reads above writes)
        Sym<1> t;
        dev::zero(t);
#pragma unroll
        for (int bb = G; bb < N; bb <<= 1)
          if (!(j & bb)) dev::xor_into(t, v[j + bb]);
        v[j] = t;
      }
      const uint8_t *wq = q.src2 + s * q.src_stride;
      const uint32_t dlw = opqu(q.dlo_log);
#pragma unroll
      for (int gg = 0; gg < G; gg++) {  // + IFFT_last(W), one group of the last IFFT phase at a time
        Sym<1> w[NI];
#pragma unroll
        for (int t = 0; t < NI; t++) {
          const uint64_t p = blk + lo + (static_cast<uint64_t>(gg + t * G) << dlw);
          if (p < q.n_src) ldp(w[t], row_rsrc(wq + p * sb), so);
          else dev::zero(w[t]);
        }
        ifft_sub<NI, 1>(w, opq(q.tabs_i), q.ti_i, q.size, q.rmax_i, 0, q.dlo_i);
#pragma unroll
        for (int t = 0; t < NI; t++) dev::xor_into(v[gg + t * G], w[t]);
        group_fence();  // one group's W rows live at a time
      }
    }
    fft_sub<N, 1>(v, q.tabs, q.ti, q.size, q.rmax, blk, q.dlo_log);
    uint8_t *y = q.dst + s * q.dst_stride;
    const uint32_t dls = opqu(q.dlo_log);
    if (acc) {
#pragma unroll
      for (int j = 0; j < N; j++) {
        const uint64_t p = blk + lo + (static_cast<uint64_t>(j) << dls);
        if (p < q.n_dst) {
          Sym<1> o;
          ldp(o, row_rsrc(y + p * sb), so);
          dev::xor_into(v[j], o);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < N; j++) {
      const uint64_t p = blk + lo + (static_cast<uint64_t>(j) << dls);
      if (act && p < q.n_dst) stp(row_rsrc(y + p * sb), so, v[j]);
    }
  }
}

// The low-rate reconstruct in block form (launch_low_blocks): the final FFT's (skew 0) first
// phase with block K's IFFT_{C, skew KC} last phase fused in (ifft_last_in), adding block K's
// share of A' = F1(U' + V) and B' = F1(U) (U = D_C's argument, U' = (I + H) U as k_dphase's
// DERIV, V the blocks' plain terms) to what the earlier blocks stored (acc): the block's
// syndromes were scaled by sigma_K, so its U term is b (u = 1) or none (u = 0) and its V term
// gamma b (the first block stores B' = 0 when it has no U term). k_dphase's LSUM then forms
// A' + L B' = F1 (D_C U + V).
template <int NI, int PASS>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3))) void k_lbfinal(uint64_t n_stripes, PhaseArgs q0, const RsTab *gamma, uint32_t u,
                                                    uint32_t acc) {
  // PASS 0: B' (u = 0: zeros, stored by the first block only); PASS 1: A' (one launch each:
  // a pass loop kept both passes' addresses live, 250+ VGPRs)
  const PhaseArgs &q = q0;
  constexpr int N = 64;
  const uint64_t sb = q.sb, uu = static_cast<uint64_t>(blockIdx.x) * kBlock + threadIdx.x;
  const bool act = uu < sb / 8;
  const uint32_t so = act ? static_cast<uint32_t>(uu * 8) : 0u;
  const uint64_t sub = blockIdx.y, dlo = 1ull << q.dlo_log;
  const uint64_t blk = (sub >> q.dlo_log) * (static_cast<uint64_t>(N) << q.dlo_log), lo = sub & (dlo - 1);
  for (uint64_t s = blockIdx.z; s < n_stripes; s += gridDim.z) {
    const PhaseArgs q = opq(q0);
    const uint8_t *x = q.src + s * q.src_stride;
    Sym<1> v[N];
#pragma unroll
    for (int j = 0; j < N; j++) {
      const uint64_t p = blk + lo + (static_cast<uint64_t>(j) << q.dlo_log);
      if (p < q.n_src && (PASS == 1 || u)) ldp(v[j], row_rsrc(x + p * sb), so);
      else dev::zero(v[j]);
    }
    ifft_last_in<N, NI>(v, q);
    if (PASS == 1 && u) {  // v = (I + H) v + gamma v, ascending (reads above writes)
      const Tab g = dev::load_tab(opq(gamma));
#pragma unroll
      for (int j = 0; j < N; j++) {
        Sym<1> t = v[j];
        dev::mul_inplace(t, g);
#pragma unroll
        for (int bb = 1; bb < N; bb <<= 1)
          if (!(j & bb)) dev::xor_into(v[j], v[j + bb]);
        dev::xor_into(v[j], t);
        group_fence();  // one product live at a time (all 64 scheduled first: 247 VGPRs)
      }
    }
    fft_sub<N, 1>(v, q.tabs, q.ti, q.size, q.rmax, blk, q.dlo_log);
    uint8_t *y = (PASS == 0 ? q.dst2 : q.dst) + s * q.dst_stride;
    const uint32_t dls = opqu(q.dlo_log);  // output offsets recomputed, not held across the transform
    if (acc) {
#pragma unroll
      for (int j = 0; j < N; j++) {
        const uint64_t p = blk + lo + (static_cast<uint64_t>(j) << dls);
        if (p < q.n_dst) {
          Sym<1> o;
          ldp(o, row_rsrc(y + p * sb), so);
          dev::xor_into(v[j], o);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < N; j++) {
      const uint64_t p = blk + lo + (static_cast<uint64_t>(j) << dls);
      if (act && p < q.n_dst) stp(row_rsrc(y + p * sb), so, v[j]);
    }
  }
}

// ======================================================= low-rate encode (§8 f4)
// The reference panics on low rate (root.zig:119-121); this is the encode of the
// algorithm it ports (rs_gf.hpp scalar_encode_low, parity unpinned): the k originals are
// positions [0, k) of one chunk C = ceilPow2(k), coefficients = IFFT(C, trunc k, skew 0),
// and recovery chunk j = FFT(coefficients, trunc min(C, m - jC), skew (j+1)C).
// Register kernel: the coefficients stay in VGPRs across the recovery chunks (each
// chunk's FFT runs on a copy), so a stripe's originals are read once and every
// recovery shard written once; twiddle tables are wave-uniform (SGPRs).
template <int C, int NV>
__global__ __launch_bounds__(kBlock) void k_encode_low_reg(EncodeArgs a) {
  uint32_t off;
  if (!lane_offset<NV>(a.shard_bytes, a.contig, off)) return;
  constexpr int TI = ifft_tabs_ce(C);
  const uint64_t sb = a.shard_bytes;
  const uint64_t s = blockIdx.y;  // launches are split at 65535 stripes
  const uint8_t *src = a.data + s * a.data_stripe_stride;
  Sym<NV> coef[C];
#pragma unroll
  for (int p = 0; p < C; p++) {
    if (static_cast<uint32_t>(p) < a.k) dev::load_sym_raw(coef[p], src + p * sb, off, a.contig);
    else dev::zero(coef[p]);
  }
#pragma unroll
  for (int p = 0; p < C; p++) dev::pair_halves(coef[p], a.contig);
  dev::ifft_regs<C>(coef, a.tabs, a.k);
  uint8_t *dst = a.parity + s * a.parity_stripe_stride;
  for (uint32_t j = 0; j < a.n_chunks; j++) {
    const uint32_t t = a.m - j * C < static_cast<uint32_t>(C) ? a.m - j * C : static_cast<uint32_t>(C);
    Sym<NV> cur[C];
#pragma unroll
    for (int p = 0; p < C; p++) cur[p] = coef[p];
    const RsTab *tj = a.tabs + TI + static_cast<uint64_t>(j) * a.tabs_per_chunk;
    asm volatile("" : "+s"(tj));  // opaque base: no per-group pointer IVs
    dev::fft_regs<C>(cur, tj, t);
    uint8_t *dj = dst + static_cast<uint64_t>(j) * C * sb;
#pragma unroll
    for (int p = 0; p < C; p++)
      if (static_cast<uint32_t>(p) < t) dev::store_sym(dj + p * sb, off, cur[p], a.contig);
  }
}

// Any C: each lane walks its column through a scratch [stripe][(1 + n_chunks) C][sb]
// (coefficients at [0, C), recovery chunk j's intermediate phases at [(1 + j) C, (2 + j) C)).
__device__ __forceinline__ uint64_t ifft_tab_count_d(uint64_t size) {
  uint64_t n = 0, d = 1, d4 = 4;
  for (; d4 <= size; d = d4, d4 <<= 2) n += 3 * (size / d4);
  return n + (d < size ? 1 : 0);
}

// Stage 1 (blockIdx.z == 0 of k_encode_low_coef): coefficients = the originals -> IFFT ->
// work[0, C) (no staging copy). Stage 2 (k_encode_low_generic, blockIdx.z = recovery chunk
// j): coefficients -> FFT (intermediate phases in work[(1 + j) C, (2 + j) C)) -> parity
// rows; the chunks run side by side (a lane's column walk is serial, so the grid's
// chunk dimension is the parallelism left at small batches).
template <int NV>
__global__ __launch_bounds__(kBlock) void k_encode_low_coef(EncodeArgs a) {
  uint32_t off;
  if (!lane_offset<NV>(a.shard_bytes, a.contig, off)) return;
  const uint64_t sb = a.shard_bytes, C = a.chunk, R = a.regions ? a.regions : 1 + a.n_chunks;
  for (uint64_t s = blockIdx.y; s < a.n_stripes; s += gridDim.y) {
    uint8_t *work = a.scratch + s * R * C * sb;
    const XformIO ic{a.data + s * a.data_stripe_stride, sb, a.k, work, sb, work, sb, C, false, false, off};
    xform_ph<NV, true>(ic, C, a.k, a.tabs);
  }
}

template <int NV>
__global__ __launch_bounds__(kBlock) void k_encode_low_generic(EncodeArgs a) {
  uint32_t off;
  if (!lane_offset<NV>(a.shard_bytes, a.contig, off)) return;
  const uint64_t sb = a.shard_bytes, C = a.chunk, TI = ifft_tab_count_d(C), j = a.chunk0 + blockIdx.z;
  const uint64_t R = a.regions ? a.regions : 1 + a.n_chunks;
  const uint64_t t = a.m - j * C < C ? a.m - j * C : C;
  for (uint64_t s = blockIdx.y; s < a.n_stripes; s += gridDim.y) {
    uint8_t *work = a.scratch + s * R * C * sb;
    uint8_t *dst = a.parity + s * a.parity_stripe_stride;
    const XformIO fc{work, sb, C, work + (1 + blockIdx.z) * C * sb, sb, dst + j * C * sb, sb, t, true, a.contig, off};
    xform_ph<NV, false>(fc, C, t, a.tabs + TI + j * a.tabs_per_chunk);
  }
}

// ================================== per-stripe erasure patterns: plans on device
// (§8f rank 2) One workgroup per stripe evaluates the erasure locator exactly as
// Generic.zig:200-215 does — FWHT truncated to chunk+k, pointwise product with
// log_walsh mod 65535, full 65536-point FWHT (walsh_hadamard.zig:16-62) — on a
// 128 KiB u16 array in LDS, then the stripe's W multiplier tables are built.
__device__ __forceinline__ uint32_t add_mod_d(uint32_t x, uint32_t y) {
  const uint32_t s = x + y;
  return (s + (s >> 16)) & 0xFFFF;
}
__device__ __forceinline__ uint32_t sub_mod_d(uint32_t x, uint32_t y) {
  const uint32_t d = x + 65535u - y;
  return (d + (d >> 16)) & 0xFFFF;
}

// walsh_hadamard.zig:16-31 over LDS, groups r < m; all threads call
__device__ void fwht_lds(uint16_t *e, uint32_t m) {
  uint32_t dist = 1;
  for (uint32_t stride = 4; stride <= 65536; dist = stride, stride *= 4) {
    const uint32_t groups = (m + stride - 1) / stride;
    const uint32_t total = groups * dist;
    for (uint32_t t = threadIdx.x; t < total; t += blockDim.x) {
      const uint32_t x0 = t / dist * stride + t % dist;
      const uint32_t x1 = x0 + dist, x2 = x1 + dist, x3 = x2 + dist;
      const uint32_t a0 = e[x0], a1 = e[x1], a2 = e[x2], a3 = e[x3];
      const uint32_t s0 = add_mod_d(a0, a1), d0 = sub_mod_d(a0, a1);
      const uint32_t s1 = add_mod_d(a2, a3), d1 = sub_mod_d(a2, a3);
      e[x0] = static_cast<uint16_t>(add_mod_d(s0, s1));
      e[x1] = static_cast<uint16_t>(add_mod_d(d0, d1));
      e[x2] = static_cast<uint16_t>(sub_mod_d(s0, s1));
      e[x3] = static_cast<uint16_t>(sub_mod_d(d0, d1));
    }
    __syncthreads();
  }
}

// per stripe: present[k+m] -> logs[W] (root.zig:277-289 + Generic.zig:200-215). low: the
// low-rate layout of rs_gf.cpp erasure_logs_low (C = ceilPow2(k): originals [0, k), known
// zeros [k, C), recovery [C, C + m), unknown [C + m, W), transform over W). A small erased set
// (W x |set| <= 2^20) is summed point by point, logs[p] = sum over erased j of log[p ^ j] mod
// 65535 (the dyadic convolution the two transforms evaluate, rs_gf.cpp erasure_logs_of: equal
// mod 65535); larger sets take the transforms in LDS.
__device__ __forceinline__ uint32_t erased_flag(const uint8_t *pr, uint32_t i, uint32_t k, uint32_t m, uint32_t C,
                                                uint32_t W, uint32_t end, uint32_t low) {
  if (low) {
    if (i < k) return pr[i] ? 0u : 1u;
    if (i >= C && i < end) return pr[k + i - C] ? 0u : 1u;
    return i >= end && i < W ? 1u : 0u;
  }
  if (i < m) return pr[k + i] ? 0u : 1u;
  if (i < C) return 1u;
  return i < end ? (pr[i - C] ? 0u : 1u) : 0u;
}

__global__ __launch_bounds__(1024) void k_erasure_logs(const uint8_t *__restrict__ present, uint64_t present_stride,
                                                       uint32_t k, uint32_t m, uint32_t C, uint32_t W, uint32_t low,
                                                       const uint16_t *__restrict__ log_walsh,
                                                       const uint16_t *__restrict__ log_t,
                                                       uint16_t *__restrict__ logs) {
  __shared__ uint16_t e[65536];
  __shared__ uint32_t n_er;
  const uint8_t *pr = present + static_cast<uint64_t>(blockIdx.x) * present_stride;
  const uint32_t end = low ? C + m : C + k, trunc = low ? W : end;
  uint16_t *out = logs + static_cast<uint64_t>(blockIdx.x) * W;
  if (threadIdx.x == 0) n_er = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < trunc; i += blockDim.x)
    if (erased_flag(pr, i, k, m, C, W, end, low)) e[atomicAdd(&n_er, 1u)] = static_cast<uint16_t>(i);
  __syncthreads();
  const uint32_t n = n_er;
  if (static_cast<uint64_t>(W) * n <= (1u << 20)) {  // integer sums: the list's order does not matter
    for (uint32_t p = threadIdx.x; p < W; p += blockDim.x) {
      uint32_t sum = 0;  // n <= 2^20 / W <= 1024 terms: no overflow
      for (uint32_t j = 0; j < n; j++) sum += log_t[p ^ e[j]];
      out[p] = static_cast<uint16_t>(sum % 65535u);
    }
    return;
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 65536; i += blockDim.x)
    e[i] = static_cast<uint16_t>(i < trunc ? erased_flag(pr, i, k, m, C, W, end, low) : 0u);
  __syncthreads();
  fwht_lds(e, trunc);
  for (uint32_t i = threadIdx.x; i < 65536; i += blockDim.x) {
    const uint32_t prod = static_cast<uint32_t>(e[i]) * log_walsh[i];
    e[i] = static_cast<uint16_t>(add_mod_d(prod & 0xFFFF, prod >> 16));
  }
  __syncthreads();
  fwht_lds(e, 65536);
  for (uint32_t p = threadIdx.x; p < W; p += blockDim.x) out[p] = e[p];
}

__device__ __forceinline__ uint32_t mul16_d(uint32_t x, uint32_t lm, const uint16_t *exp, const uint16_t *log) {
  return x == 0 ? 0 : exp[add_mod_d(log[x], lm)];
}
__device__ uint32_t mul_engine_d(uint32_t x, uint32_t lm, bool d1, const uint16_t *exp, const uint16_t *log) {
  if (!d1) return mul16_d(x, lm, exp, log);
  const uint32_t xh = ((x & 0xF) << 4) ^ (x & 0xFFF0);
  return (mul16_d(x, lm, exp, log) & 0xFF) | (mul16_d(xh, lm, exp, log) & 0xFF00);
}
// rs_gf.cpp make_tab on device
__device__ void make_tab_d(RsTab &t, uint32_t lm, bool d1, const uint16_t *exp, const uint16_t *log) {
  constexpr int kOff[6] = {0, 3, 6, 8, 11, 14};
  constexpr int kBits[6] = {3, 3, 2, 3, 3, 2};
  constexpr int kSlot[6] = {0, 2, 4, 5, 7, 9};
#pragma unroll
  for (int i = 0; i < 10; i++) t.lo[i] = t.hi[i] = 0;
#pragma unroll
  for (int f = 0; f < 6; f++)
    for (uint32_t v = 0; v < (1u << kBits[f]); v++) {
      const uint32_t p = mul_engine_d(v << kOff[f], lm, d1, exp, log);
      const int w = kSlot[f] + (v >> 2), sh = 8 * (v & 3);
      t.lo[w] |= (p & 0xFF) << sh;
      t.hi[w] |= (p >> 8) << sh;
    }
  t.flags = 0;
  t.log_m = lm;
  t.pad[0] = t.pad[1] = 0;
}

// per (stripe, position): masks, sources, restored slots (root.zig:291-326)
__global__ __launch_bounds__(256) void k_pattern_tables(const uint8_t *__restrict__ present, uint64_t present_stride,
                                                        uint32_t k, uint32_t m, uint32_t C, uint32_t W, uint32_t n,
                                                        uint32_t max_e, bool d1, uint32_t low,
                                                        const uint16_t *__restrict__ logs,
                                                        const uint16_t *__restrict__ exp, const uint16_t *__restrict__ log,
                                                        RsTab *pre, RsTab *post, int32_t *src, int32_t *dst,
                                                        int32_t *status) {
  const uint64_t g = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g >= static_cast<uint64_t>(n) * W) return;
  const uint64_t s = g / W;
  const uint32_t p = static_cast<uint32_t>(g % W);
  const uint8_t *pr = present + s * present_stride;
  if (p == 0 && status) {  // root.zig:271 NotEnoughShards; restored slots beyond max_e: InvalidArgument
    uint32_t have = 0, e = 0;
    for (uint32_t i = 0; i < k + m; i++) have += pr[i] ? 1 : 0;
    for (uint32_t i = 0; i < k; i++) e += pr[i] ? 0 : 1;
    status[s] = have < k ? 2 : (e > max_e ? 14 : 0);
  }
  const uint32_t lm = logs[g];
  int32_t sv = -1, dv = -1;
  RsTab tp{}, tq{};
  // positions: originals at o0 + i, recovery at r0 + r (low rate: o0 = 0, r0 = C)
  const uint32_t o0 = low ? 0 : C, r0 = low ? C : 0;
  if (p >= r0 && p < r0 + m && pr[k + p - r0]) {
    sv = kSrcRecovery | static_cast<int32_t>(p - r0);
    make_tab_d(tp, lm, d1, exp, log);
  } else if (p >= o0 && p < o0 + k && pr[p - o0]) {
    sv = static_cast<int32_t>(p - o0);
    make_tab_d(tp, lm, d1, exp, log);
  }
  if (p >= o0 && p < o0 + k && !pr[p - o0]) {
    int32_t slot = 0;
    for (uint32_t i = 0; i < p - o0; i++) slot += pr[i] ? 0 : 1;
    dv = slot < static_cast<int32_t>(max_e) ? slot : -1;
    make_tab_d(tq, 65535u - lm, d1, exp, log);
  }
  pre[g] = tp;
  post[g] = tq;
  src[g] = sv;
  dst[g] = dv;
}

// ---- per-stripe patterns as per-stripe e x k matrices (corrected multiply)
// One thread per (stripe, input t, basis bit b): the reconstruct of root.zig:268-335
// on one symbol per position (W <= 32 in registers), input t = basis symbol 1 << b,
// every other position zero; the restored originals are column (t, b) of the
// stripe's map. Inputs: the present originals, then the first e present recovery
// shards (k in all); outputs: the missing originals, ascending, up to max_e.
__device__ __forceinline__ void ifft_bf_s(uint32_t &x, uint32_t &y, const RsTab &t, const uint16_t *exp,
                                          const uint16_t *log) {
  y ^= x;
  if (!(t.flags & kTabXorOnly)) x ^= mul16_d(y, t.log_m, exp, log);
}
__device__ __forceinline__ void fft_bf_s(uint32_t &x, uint32_t &y, const RsTab &t, const uint16_t *exp,
                                         const uint16_t *log) {
  if (!(t.flags & kTabXorOnly)) x ^= mul16_d(y, t.log_m, exp, log);
  y ^= x;
}

template <int W>
__global__ __launch_bounds__(256) void k_pattern_images(const uint8_t *__restrict__ present, uint64_t present_stride,
                                                        uint32_t k, uint32_t m, uint32_t C, uint64_t n, uint32_t max_e,
                                                        const uint16_t *__restrict__ logs, const RsTab *__restrict__ ti,
                                                        const RsTab *__restrict__ tf, const uint16_t *__restrict__ exp,
                                                        const uint16_t *__restrict__ log, uint16_t *__restrict__ images,
                                                        int32_t *__restrict__ srcs, int32_t *__restrict__ nout) {
  const uint64_t g = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g >= n * k * 16) return;
  const uint64_t s = g / (k * 16);
  const uint32_t t = static_cast<uint32_t>(g / 16 % k), b = static_cast<uint32_t>(g % 16);
  const uint8_t *pr = present + s * present_stride;
  const uint16_t *lg = logs + s * W;
  uint32_t have = 0, e = 0;
  for (uint32_t i = 0; i < k + m; i++) have += pr[i] ? 1 : 0;
  for (uint32_t i = 0; i < k; i++) e += pr[i] ? 0 : 1;
  int32_t in_pos = -1, src = 0;
  uint32_t cnt = 0;
  for (uint32_t i = 0; i < k && in_pos < 0; i++)
    if (pr[i]) {
      if (cnt == t) in_pos = static_cast<int32_t>(C + i), src = static_cast<int32_t>(i);
      cnt++;
    }
  for (uint32_t r = 0; r < m && in_pos < 0; r++)
    if (pr[k + r]) {
      if (cnt == t) in_pos = static_cast<int32_t>(r), src = kSrcRecovery | static_cast<int32_t>(r);
      cnt++;
    }
  if (b == 0) srcs[s * k + t] = src;  // a valid shard even for NotEnoughShards stripes (nothing is stored)
  if (t == 0 && b == 0) nout[s] = have >= k ? static_cast<int32_t>(min(e, max_e)) : 0;
  const uint32_t trunc = C + k;
  uint32_t v[W];
  const uint32_t x0 = in_pos >= 0 ? mul16_d(1u << b, lg[in_pos], exp, log) : 0u;  // erasure mask, root.zig:291-302
#pragma unroll
  for (int p = 0; p < W; p++) v[p] = p == in_pos ? x0 : 0u;
  {  // IFFT, Generic.zig:80-147 (schedule of push_ifft_tabs)
    int q = 0, d = 1;
#pragma unroll
    for (int d4 = 4; d4 <= W; d4 <<= 2) {
#pragma unroll
      for (int r = 0; r < W; r += d4) {
        if (static_cast<uint32_t>(r) < trunc) {
          const RsTab m01 = ti[q], m02 = ti[q + 1], m23 = ti[q + 2];
#pragma unroll
          for (int i = r; i < r + d; i++) {
            ifft_bf_s(v[i], v[i + d], m01, exp, log);
            ifft_bf_s(v[i + 2 * d], v[i + 3 * d], m23, exp, log);
            ifft_bf_s(v[i], v[i + 2 * d], m02, exp, log);
            ifft_bf_s(v[i + d], v[i + 3 * d], m02, exp, log);
          }
        }
        q += 3;
      }
      d = d4;
    }
    if (d < W) {
#pragma unroll
      for (int i = 0; i < d; i++) ifft_bf_s(v[i], v[d + i], ti[q], exp, log);
    }
  }
#pragma unroll
  for (int i = 1; i < W; i++) {  // formal derivative, root.zig:309-315
    const int w = i & -i;
#pragma unroll
    for (int j = 0; j < w; j++)
      if (i + j < W) v[i - w + j] ^= v[i + j];
  }
  {  // FFT, Generic.zig:15-78 (schedule of push_fft_tabs)
    int q = 0, d4 = W;
#pragma unroll
    for (int d = W >> 2; d != 0; d >>= 2) {
#pragma unroll
      for (int r = 0; r < W; r += d4) {
        if (static_cast<uint32_t>(r) < trunc) {
          const RsTab m01 = tf[q], m02 = tf[q + 1], m23 = tf[q + 2];
#pragma unroll
          for (int i = r; i < r + d; i++) {
            fft_bf_s(v[i], v[i + 2 * d], m02, exp, log);
            fft_bf_s(v[i + d], v[i + 3 * d], m02, exp, log);
            fft_bf_s(v[i], v[i + d], m01, exp, log);
            fft_bf_s(v[i + 2 * d], v[i + 3 * d], m23, exp, log);
          }
        }
        q += 3;
      }
      d4 = d;
    }
    if (d4 == 2) {
#pragma unroll
      for (int r = 0; r < W; r += 2)
        if (static_cast<uint32_t>(r) < trunc) fft_bf_s(v[r], v[r + 1], tf[q + r / 2], exp, log);
    }
  }
  uint16_t *img = images + (s * k + t) * max_e * 16 + b;
  uint32_t j = 0;
#pragma unroll
  for (int p = 0; p < W; p++) {  // reveal the missing originals, root.zig:320-326
    if (static_cast<uint32_t>(p) >= C && static_cast<uint32_t>(p) < C + k && !pr[p - C]) {
      if (j < max_e) img[j * 16] = static_cast<uint16_t>(mul16_d(v[p], 65535u - lg[p], exp, log));
      j++;
    }
  }
  for (; j < max_e; j++) img[j * 16] = 0;
}

// Per-stripe plan of the syndrome-network path (rs_psyn.hpp), one thread per stripe:
// E = the erased originals, R = the first e present recovery rows, A = G[R][E] (e x e
// block of the code's encode coefficients, G[r][t] = parity r of data t = 1), and
// x_E = A^-1 s_R with s_r = p_r ^ Enc_r(data, erased read as 0). Block per stripe
// (u32, nw = ceil(k / 32)): [0, nw) erased mask, [nw] R mask, [nw + 1] outputs stored =
// min(e, max_e) (0: none), then [nw + 2 + r * max_out + j] = A^-1[j][i(r)] in polynomial
// coordinates (bit i: the coefficient of alpha^i; 0 for rows outside R), the form the
// kernel multiplies in.
// G: [m][k] coefficients followed by the 16 Cantor basis elements (polynomial form).
__device__ __forceinline__ uint32_t gf_mul_d(uint32_t a, uint32_t b, const uint16_t *exp, const uint16_t *log) {
  return (a == 0 || b == 0) ? 0u : exp[add_mod_d(log[a], log[b])];
}

__global__ __launch_bounds__(64) void k_psyn_plan(const uint8_t *__restrict__ present, uint64_t present_stride,
                                                  uint32_t k, uint32_t m, uint32_t max_out, uint32_t max_e, uint64_t n,
                                                  const uint16_t *__restrict__ G, const uint16_t *__restrict__ exp,
                                                  const uint16_t *__restrict__ log, uint32_t *__restrict__ plan,
                                                  uint32_t plan_dw, int32_t *__restrict__ status) {
  const uint64_t s = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const uint8_t *pr = present + s * present_stride;
  uint32_t *pl = plan + s * plan_dw;
  const uint32_t nw = (k + 31) / 32;  // erased-original mask words (rs_psyn.hpp plan_dwords)
  uint32_t have = 0, e = 0;
  for (uint32_t i = 0; i < k + m; i++) have += pr[i] ? 1 : 0;
  for (uint32_t i = 0; i < k; i++) e += pr[i] ? 0 : 1;
  if (status) status[s] = have < k ? 2 : (e > max_e ? 14 : 0);  // as k_pattern_tables
  for (uint32_t w = 0; w < nw + 2; w++) pl[w] = 0;
  if (have < k || e == 0) return;  // nothing restored (e <= present recovery <= m from here)
  uint32_t E[kPsynMaxM], R[kPsynMaxM], rm = 0;
  for (uint32_t i = 0, c = 0; i < k && c < e; i++)
    if (!pr[i]) E[c++] = i;
  for (uint32_t r = 0, c = 0; r < m && c < e; r++)
    if (pr[k + r]) R[c++] = r, rm |= 1u << r;
  // Gauss-Jordan on [A | I] over GF(2^16)
  uint32_t A[kPsynMaxM][2 * kPsynMaxM];
  for (uint32_t i = 0; i < e; i++)
    for (uint32_t j = 0; j < 2 * e; j++) A[i][j] = j < e ? G[R[i] * k + E[j]] : (j - e == i ? 1u : 0u);
  for (uint32_t c = 0; c < e; c++) {
    uint32_t piv = c;
    while (piv < e && A[piv][c] == 0) piv++;
    if (piv == e) {  // singular: not an MDS code (the host keeps such codes off this path)
      if (status) status[s] = 15;  // RS_ERR_DEVICE: nothing restored
      return;
    }
    for (uint32_t j = 0; j < 2 * e; j++) {
      const uint32_t t = A[c][j];
      A[c][j] = A[piv][j];
      A[piv][j] = t;
    }
    const uint32_t inv = exp[(65535u - log[A[c][c]]) % 65535u];
    for (uint32_t j = 0; j < 2 * e; j++) A[c][j] = gf_mul_d(A[c][j], inv, exp, log);
    for (uint32_t i = 0; i < e; i++)
      if (i != c && A[i][c]) {
        const uint32_t f = A[i][c];
        for (uint32_t j = 0; j < 2 * e; j++) A[i][j] ^= gf_mul_d(f, A[c][j], exp, log);
      }
  }
  const uint16_t *cantor = G + m * k;
  for (uint32_t r = 0; r < m; r++) {
    int32_t ir = -1;
    for (uint32_t i = 0; i < e; i++) ir = R[i] == r ? static_cast<int32_t>(i) : ir;
    for (uint32_t j = 0; j < max_out; j++) {
      const uint32_t c = (ir >= 0 && j < e) ? A[j][e + ir] : 0u;  // x_j += A^-1[j][i] s_{R_i}
      uint32_t poly = 0;
      for (int b = 0; b < 16; b++) poly ^= (c >> b & 1u) ? cantor[b] : 0u;
      pl[nw + 2 + r * max_out + j] = poly;
    }
  }
  for (uint32_t i = 0; i < e; i++) pl[E[i] / 32] |= 1u << (E[i] % 32);
  pl[nw] = rm;
  pl[nw + 1] = e < max_e ? e : max_e;
}

// Per-stripe plan of the wide-code path (rs_psyn.hpp solve kernel after the FFT
// syndrome kernel, chunk 32 / 64): as k_psyn_plan for any e <= m <= 64, one thread per
// stripe (the e x 2e Gauss-Jordan lives in private memory). Block per stripe (u32):
// [0, dmw) the FFT kernel's masks (fftnet::dyn_mask_words: erased data bits, then the
// R rows stored), then at hdr = dmw: [0] outputs stored = min(e, max_e), [1] e,
// [2, 2 + 64) R, [66 + i * cs + j] = A^-1[j][i] in polynomial form for j < cs
// (cs = wps_coef_stride(max_e): 8, or max_e rounded up to 8 for the wave kernel below).
constexpr uint32_t kWpsMaxM = 64, kWpsMaxOut = 8;
__global__ __launch_bounds__(64) void k_wps_plan(const uint8_t *__restrict__ present, uint64_t present_stride,
                                                 uint32_t k, uint32_t m, uint32_t max_e, uint64_t n,
                                                 const uint16_t *__restrict__ G, const uint16_t *__restrict__ exp,
                                                 const uint16_t *__restrict__ log, uint32_t *__restrict__ plan,
                                                 uint32_t plan_dw, uint32_t dmw, int32_t *__restrict__ status) {
  const uint64_t s = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const uint8_t *pr = present + s * present_stride;
  uint32_t *pl = plan + s * plan_dw, *hd = pl + dmw;
  uint32_t have = 0, e = 0;
  for (uint32_t i = 0; i < k + m; i++) have += pr[i] ? 1 : 0;
  for (uint32_t i = 0; i < k; i++) e += pr[i] ? 0 : 1;
  if (status) status[s] = have < k ? 2 : (e > max_e ? 14 : 0);  // as k_pattern_tables
  for (uint32_t i = 0; i < dmw; i++) pl[i] = 0;
  hd[0] = hd[1] = 0;
  if (have < k || e == 0) return;
  uint16_t E[kWpsMaxM], R[kWpsMaxM];
  for (uint32_t i = 0, c = 0; i < k && c < e; i++)
    if (!pr[i]) E[c++] = static_cast<uint16_t>(i);
  for (uint32_t r = 0, c = 0; r < m && c < e; r++)
    if (pr[k + r]) R[c++] = static_cast<uint16_t>(r);
  uint16_t A[kWpsMaxM][2 * kWpsMaxM];
  for (uint32_t i = 0; i < e; i++)
    for (uint32_t j = 0; j < 2 * e; j++)
      A[i][j] = static_cast<uint16_t>(j < e ? G[R[i] * k + E[j]] : (j - e == i ? 1u : 0u));
  for (uint32_t c = 0; c < e; c++) {
    uint32_t piv = c;
    while (piv < e && A[piv][c] == 0) piv++;
    if (piv == e) {  // singular: not an MDS code (the host keeps such codes off this path)
      if (status) status[s] = 15;  // RS_ERR_DEVICE: nothing restored
      hd[0] = 0;
      return;
    }
    for (uint32_t j = 0; j < 2 * e; j++) {
      const uint16_t t = A[c][j];
      A[c][j] = A[piv][j];
      A[piv][j] = t;
    }
    const uint32_t inv = exp[(65535u - log[A[c][c]]) % 65535u];
    for (uint32_t j = c; j < 2 * e; j++) A[c][j] = static_cast<uint16_t>(gf_mul_d(A[c][j], inv, exp, log));
    for (uint32_t i = 0; i < e; i++)
      if (i != c && A[i][c]) {
        const uint32_t f = A[i][c];
        for (uint32_t j = c; j < 2 * e; j++) A[i][j] ^= static_cast<uint16_t>(gf_mul_d(f, A[c][j], exp, log));
      }
  }
  const uint16_t *cantor = G + m * k;
  const uint32_t kw = dmw - 2;  // skip words, then 2 store words
  for (uint32_t i = 0; i < e; i++) {
    pl[E[i] / 32] |= 1u << (E[i] % 32);
    pl[kw + R[i] / 32] |= 1u << (R[i] % 32);
    hd[2 + i] = R[i];
    for (uint32_t j = 0; j < kWpsMaxOut; j++) {
      const uint32_t c = j < e ? A[j][e + i] : 0u;
      uint32_t poly = 0;
      for (int b = 0; b < 16; b++) poly ^= (c >> b & 1u) ? cantor[b] : 0u;
      hd[2 + kWpsMaxM + i * kWpsMaxOut + j] = poly;
    }
  }
  hd[1] = e;
  hd[0] = e < max_e ? e : max_e;
}

// The same plan for max_e > 8 (every output of up to 64 erased originals): one wave per
// stripe, the e x 2e Gauss-Jordan in LDS with the columns spread over the lanes (a
// thread per stripe would run e^3 / 3 table multiplies on its own: ~55,000 for e = 55).
// Coefficients at [66 + i * cs + j] for j < cs (cs = max_e rounded up to 8, <= 64).
__global__ __launch_bounds__(64) void k_wps_plan_wave(const uint8_t *__restrict__ present, uint64_t present_stride,
                                                      uint32_t k, uint32_t m, uint32_t max_e,
                                                      const uint16_t *__restrict__ G, const uint16_t *__restrict__ exp,
                                                      const uint16_t *__restrict__ log, uint32_t *__restrict__ plan,
                                                      uint32_t plan_dw, uint32_t dmw, uint32_t cs,
                                                      int32_t *__restrict__ status) {
  __shared__ uint16_t A[kWpsMaxM][2 * kWpsMaxM];
  __shared__ uint16_t E[kWpsMaxM], R[kWpsMaxM];
  const uint64_t s = blockIdx.x;
  const uint32_t t = threadIdx.x;
  const uint8_t *pr = present + s * present_stride;
  uint32_t *pl = plan + s * plan_dw, *hd = pl + dmw;
  uint32_t have = 0, e = 0;
  for (uint32_t i = t; i < k + m; i += 64) {
    have += pr[i] ? 1u : 0u;
    e += (i < k && !pr[i]) ? 1u : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) {
    have += __shfl_xor(have, o);
    e += __shfl_xor(e, o);
  }
  if (t == 0 && status) status[s] = have < k ? 2 : (e > max_e ? 14 : 0);  // as k_pattern_tables
  for (uint32_t i = t; i < dmw; i += 64) pl[i] = 0;
  if (t == 0) hd[0] = hd[1] = 0;
  if (have < k || e == 0 || e > kWpsMaxM) return;  // wave-uniform
  if (t == 0) {
    for (uint32_t i = 0, c = 0; i < k && c < e; i++)
      if (!pr[i]) E[c++] = static_cast<uint16_t>(i);
    for (uint32_t r = 0, c = 0; r < m && c < e; r++)
      if (pr[k + r]) R[c++] = static_cast<uint16_t>(r);
  }
  __syncthreads();
  for (uint32_t i = 0; i < e; i++)
    for (uint32_t j = t; j < 2 * e; j += 64)
      A[i][j] = static_cast<uint16_t>(j < e ? G[R[i] * k + E[j]] : (j - e == i ? 1u : 0u));
  __syncthreads();
  for (uint32_t c = 0; c < e; c++) {
    const uint64_t nz = __ballot(t >= c && t < e && A[t][c] != 0);
    if (nz == 0) {  // singular: not an MDS code (the host keeps such codes off this path)
      if (t == 0 && status) status[s] = 15;  // RS_ERR_DEVICE: nothing restored
      if (t == 0) hd[0] = 0;
      return;
    }
    const uint32_t piv = static_cast<uint32_t>(__ffsll(static_cast<unsigned long long>(nz)) - 1);
    if (piv != c)
      for (uint32_t j = t; j < 2 * e; j += 64) {
        const uint16_t x = A[c][j];
        A[c][j] = A[piv][j];
        A[piv][j] = x;
      }
    __syncthreads();
    const uint32_t inv = exp[(65535u - log[A[c][c]]) % 65535u];
    __syncthreads();  // every lane has read the pivot before its column is scaled
    for (uint32_t j = t; j < 2 * e; j += 64) A[c][j] = static_cast<uint16_t>(gf_mul_d(A[c][j], inv, exp, log));
    __syncthreads();
    // elimination: lane t owns columns t and t + 64 and holds row t's factor; the logs of
    // the pivot row's entries are looked up once per pivot, so each update is one
    // independent exp lookup (no dependent table chain, no barrier per row)
    const uint32_t fr = t < e ? A[t][c] : 0u, lfr = fr ? log[fr] : 0u;
    const uint32_t p0 = t < 2 * e ? A[c][t] : 0u, p1 = t + 64 < 2 * e ? A[c][t + 64] : 0u;
    const uint32_t lp0 = p0 ? log[p0] : 0u, lp1 = p1 ? log[p1] : 0u;
    __syncthreads();  // column c read by every lane before its owner rewrites it
#pragma unroll 4
    for (uint32_t i = 0; i < e; i++) {
      const uint32_t f = __shfl(fr, static_cast<int>(i)), lf = __shfl(lfr, static_cast<int>(i));
      if (i == c || f == 0) continue;  // wave-uniform
      if (p0) A[i][t] ^= exp[add_mod_d(lf, lp0)];
      if (p1) A[i][t + 64] ^= exp[add_mod_d(lf, lp1)];
    }
    __syncthreads();
  }
  const uint16_t *cantor = G + m * k;
  const uint32_t kw = dmw - 2;  // skip words, then 2 store words
  if (t == 0)
    for (uint32_t i = 0; i < e; i++) {
      pl[E[i] / 32] |= 1u << (E[i] % 32);
      pl[kw + R[i] / 32] |= 1u << (R[i] % 32);
    }
  for (uint32_t i = t; i < e; i += 64) hd[2 + i] = R[i];
  for (uint32_t x = t; x < e * cs; x += 64) {
    const uint32_t i = x / cs, j = x % cs;
    const uint32_t c = j < e ? A[j][e + i] : 0u;
    uint32_t poly = 0;
    for (int b = 0; b < 16; b++) poly ^= (c >> b & 1u) ? cantor[b] : 0u;
    hd[2 + kWpsMaxM + i * cs + j] = poly;
  }
  if (t == 0) {
    hd[1] = e;
    hd[0] = e < max_e ? e : max_e;
  }
}

// The matrix path decodes from exactly k received shards (the present originals and
// the first e present recovery shards), so the erasure locator must be evaluated for
// that set: present rows with the other recovery shards marked absent.
__global__ __launch_bounds__(256) void k_trim_present(const uint8_t *__restrict__ present, uint64_t present_stride,
                                                      uint32_t k, uint32_t m, uint64_t n, uint8_t *__restrict__ out) {
  const uint64_t s = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (s >= n) return;
  const uint8_t *pr = present + s * present_stride;
  uint8_t *o = out + s * (k + m);
  uint32_t e = 0;
  for (uint32_t i = 0; i < k; i++) {
    o[i] = pr[i] ? 1 : 0;
    e += pr[i] ? 0 : 1;
  }
  uint32_t used = 0;
  for (uint32_t r = 0; r < m; r++) {
    const bool keep = pr[k + r] && used < e;
    used += keep ? 1 : 0;
    o[k + r] = keep ? 1 : 0;
  }
  // fewer than k present in total: keep the row as it is (the plan reports NotEnoughShards)
  if (used < e)
    for (uint32_t r = 0; r < m; r++) o[k + r] = pr[k + r] ? 1 : 0;
}

// rs_gf.cpp make_tab_from_images on device: one thread per (stripe, input, output)
__global__ __launch_bounds__(256) void k_pattern_mtabs(const uint16_t *__restrict__ images, uint64_t count,
                                                       RsTab *__restrict__ tabs) {
  const uint64_t g = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g >= count) return;
  const uint16_t *img = images + g * 16;
  constexpr int kOff[6] = {0, 3, 6, 8, 11, 14};
  constexpr int kBits[6] = {3, 3, 2, 3, 3, 2};
  constexpr int kSlot[6] = {0, 2, 4, 5, 7, 9};
  RsTab t;
#pragma unroll
  for (int i = 0; i < 10; i++) t.lo[i] = t.hi[i] = 0;
#pragma unroll
  for (int f = 0; f < 6; f++)
    for (uint32_t v = 0; v < (1u << kBits[f]); v++) {
      uint32_t p = 0;
      for (int bit = 0; bit < kBits[f]; bit++)
        if (v >> bit & 1) p ^= img[kOff[f] + bit];
      const int w = kSlot[f] + (v >> 2), sh = 8 * (v & 3);
      t.lo[w] |= (p & 0xFF) << sh;
      t.hi[w] |= (p >> 8) << sh;
    }
  t.flags = 0;
  t.log_m = 0;
  t.pad[0] = t.pad[1] = 0;
  tabs[g] = t;
}

hipError_t launch_pattern_matrix_impl(const uint8_t *d_present, uint64_t present_stride, uint32_t k, uint32_t m,
                                      uint32_t C, uint32_t W, uint64_t n, uint32_t max_e, const uint16_t *logs,
                                      const RsTab *tab_ifft, const RsTab *tab_fft, const uint16_t *d_exp,
                                      const uint16_t *d_log, uint16_t *images, RsTab *tabs, int32_t *srcs,
                                      int32_t *nout, hipStream_t s) {
  const uint64_t threads = n * k * 16;
  const dim3 grid(static_cast<uint32_t>((threads + 255) / 256));
  trace_launch("k_pattern_images");
  trace_launch("k_pattern_mtabs");
  switch (W) {
#define RS_PIMG(W_)                                                                                                   \
  case W_:                                                                                                            \
    hipLaunchKernelGGL(k_pattern_images<W_>, grid, dim3(256), 0, s, d_present, present_stride, k, m, C, n, max_e, logs, \
                       tab_ifft, tab_fft, d_exp, d_log, images, srcs, nout);                                          \
    break;
    RS_PIMG(2) RS_PIMG(4) RS_PIMG(8) RS_PIMG(16) RS_PIMG(32)
#undef RS_PIMG
    default: return hipErrorInvalidValue;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const uint64_t count = n * k * max_e;
  hipLaunchKernelGGL(k_pattern_mtabs, dim3(static_cast<uint32_t>((count + 255) / 256)), dim3(256), 0, s, images, count,
                     tabs);
  return hipGetLastError();
}

hipError_t launch_pattern_plan_impl(const uint8_t *d_present, uint64_t present_stride, uint32_t k, uint32_t m,
                                    uint32_t C, uint32_t W, uint64_t n, uint32_t max_e, bool d1, bool low,
                                    const uint16_t *d_exp, const uint16_t *d_log, const uint16_t *d_log_walsh,
                                    uint16_t *logs, RsTab *pre,
                                    RsTab *post, int32_t *src, int32_t *dst, int32_t *status, hipStream_t s) {
  trace_launch("k_erasure_logs");
  trace_launch("k_pattern_tables");
  for (uint64_t s0 = 0; s0 < n; s0 += 65535) {
    const uint32_t cnt = static_cast<uint32_t>(std::min<uint64_t>(65535, n - s0));
    hipLaunchKernelGGL(k_erasure_logs, dim3(cnt), dim3(1024), 0, s, d_present + s0 * present_stride,
                       present_stride, k, m, C, W, low ? 1u : 0u, d_log_walsh, d_log, logs + s0 * W);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const uint64_t total = n * W;
  const uint64_t blocks = (total + 255) / 256;
  hipLaunchKernelGGL(k_pattern_tables, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, d_present,
                     present_stride, k, m, C, W, static_cast<uint32_t>(n), max_e, d1, low ? 1u : 0u, logs, d_exp, d_log,
                     pre, post,
                     src, dst, status);
  return hipGetLastError();
}

// ======================================================= shard tails (sb % 64)
// The reference panics on tails (root.zig:385); its undoLastChunkEncoding
// (root.zig:338-348) implies the layout: a tail of t bytes is coded as one more
// chunk with bytes [0,t/2) as lo bytes [0,t/2) and [t/2,t) as hi bytes
// [32,32+t/2). Pack/unpack one shard's tail chunk for n stripes (one thread per
// byte of the 64-B chunk); whole chunks are moved with hipMemcpy2DAsync.
__global__ __launch_bounds__(256) void k_tail_pack(const uint8_t *__restrict__ src, uint64_t src_stripe_stride,
                                                   uint8_t *__restrict__ dst, uint64_t dst_stripe_stride,
                                                   uint64_t sb, uint64_t n, int unpack) {
  const uint64_t g = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (g >= n * 64) return;
  const uint64_t s = g / 64;
  const uint32_t j = static_cast<uint32_t>(g % 64);
  const uint32_t t = static_cast<uint32_t>(sb % 64), h = t / 2;
  const uint64_t whole = sb - t;
  if (!unpack) {  // real shard (sb bytes) -> padded tail chunk
    const uint8_t *in = src + s * src_stripe_stride + whole;
    uint8_t v = 0;
    if (j < h) v = in[j];
    else if (j >= 32 && j < 32 + h) v = in[h + j - 32];
    dst[s * dst_stripe_stride + whole + j] = v;
  } else if (j < t) {  // padded tail chunk -> real shard
    const uint8_t *in = src + s * src_stripe_stride + whole;
    dst[s * dst_stripe_stride + whole + j] = j < h ? in[j] : in[32 + j - h];
  }
}

// ========================================================== engine test shims
__global__ __launch_bounds__(kBlock) void k_engine_transform(uint8_t *work, uint64_t sb, uint64_t pos, uint64_t size,
                                                             uint64_t trunc, const RsTab *tabs, int inverse) {
  uint32_t off;
  if (!lane_offset<1>(sb, false, off)) return;
  if (inverse) ifft_mem<1>(work + pos * sb, off, sb, size, trunc, tabs);
  else fft_mem<1>(work + pos * sb, off, sb, size, trunc, tabs);
}

__global__ __launch_bounds__(kBlock) void k_mul_scalar(uint8_t *chunks, uint64_t bytes, const RsTab *tab) {
  uint32_t off;
  if (!lane_offset<1>(bytes, false, off)) return;
  Sym<1> v;
  ld(v, chunks + off);
  dev::mul_inplace(v, dev::load_tab(tab));
  st(chunks + off, v);
}

dim3 grid_for(uint64_t shard_bytes, int nv, uint64_t n_stripes) {
  const uint64_t units = shard_bytes / 64 * (8 / nv);
  const uint64_t bx = (units + kBlock - 1) / kBlock;
  const uint64_t by = n_stripes < 65535 ? n_stripes : 65535;
  return dim3(static_cast<uint32_t>(bx), static_cast<uint32_t>(by ? by : 1), 1);
}

}  // namespace

// ---------------------------------------------------------------- selection
// Instantiated register variants (see launch_*): encode keeps acc + one chunk
// (2*C slots) live with 2*C*2*NV <= 64 VGPRs of state; decode keeps W slots,
// W*2*NV <= 128.
static int clamp_nv(int nv, int size, bool enc) {
  const int live = enc ? 2 * size : size;  // symbol slots live at once
  const int limit = enc ? 64 : 128;
  while (nv > 1 && live * 2 * nv > limit) nv >>= 1;
  return nv;
}

// A wave of the register / matrix kernels covers 512 * NV bytes of a shard: when
// that leaves more than 1/8 of the lanes idle (small shards), halve NV.
// RS(32,32) 1 KiB x 65536, 4 erased: decode_matrix_e4 nv4 1.43 -> nv1 0.97 ms.
static int fit_nv(int nv, uint64_t shard_bytes) {
  while (nv > 1) {
    const uint64_t w = 512ull * nv, idle = (shard_bytes + w - 1) / w * w - shard_bytes;
    if (idle * 8 <= shard_bytes) break;
    nv >>= 1;
  }
  return nv;
}

static int env_nv(int dflt) {
  const char *e = getenv("RS_AMD_NV");
  if (!e) return dflt;
  const int v = atoi(e);
  return (v == 1 || v == 2 || v == 4) ? v : dflt;
}

static const char *reg_name(bool enc, int size, int nv) {
  static const char *kEnc[6][3] = {
      {"encode_reg_w1_nv1", "encode_reg_w1_nv2", "encode_reg_w1_nv4"},
      {"encode_reg_w2_nv1", "encode_reg_w2_nv2", "encode_reg_w2_nv4"},
      {"encode_reg_w4_nv1", "encode_reg_w4_nv2", "encode_reg_w4_nv4"},
      {"encode_reg_w8_nv1", "encode_reg_w8_nv2", "encode_reg_w8_nv4"},
      {"encode_reg_w16_nv1", "encode_reg_w16_nv2", "encode_reg_w16_nv4"},
      {"encode_reg_w32_nv1", "encode_reg_w32_nv2", "encode_reg_w32_nv4"}};
  static const char *kDec[6][3] = {
      {"decode_reg_w1_nv1", "decode_reg_w1_nv2", "decode_reg_w1_nv4"},
      {"decode_reg_w2_nv1", "decode_reg_w2_nv2", "decode_reg_w2_nv4"},
      {"decode_reg_w4_nv1", "decode_reg_w4_nv2", "decode_reg_w4_nv4"},
      {"decode_reg_w8_nv1", "decode_reg_w8_nv2", "decode_reg_w8_nv4"},
      {"decode_reg_w16_nv1", "decode_reg_w16_nv2", "decode_reg_w16_nv4"},
      {"decode_reg_w32_nv1", "decode_reg_w32_nv2", "decode_reg_w32_nv4"}};
  int si = 0;
  while ((1 << si) < size) si++;
  const int ni = nv == 1 ? 0 : nv == 2 ? 1 : 2;
  return enc ? kEnc[si][ni] : kDec[si][ni];
}

KernelChoice choose_encode(uint64_t k, uint64_t m, uint64_t shard_bytes, int max_nv) {
  (void)k;
  const uint64_t C = ceil_pow2(m);
  if (C <= 32) {  // C = 32: 64 live slots of one dword pair (NV = 1)
    const int c = static_cast<int>(C);
    const int nv = clamp_nv(fit_nv(std::min(env_nv(4), max_nv), shard_bytes), c, true);
    return {Variant::kRegister, c, nv, reg_name(true, c, nv)};
  }
  if (C == 64 && shard_bytes % 512 == 0) {
    int nv = std::min(std::min(env_nv(1), max_nv), 2);
    if (shard_bytes % (512 * nv)) nv = 1;  // whole 64-lane regions only
    return {Variant::kWaveSplit, 64, nv, nv == 1 ? "encode_ws64_nv1" : "encode_ws64_nv2"};
  }
  return {Variant::kGeneric, static_cast<int>(C), 1, "encode_generic_nv1"};
}

KernelChoice choose_decode(uint64_t k, uint64_t m, uint64_t shard_bytes, int max_nv) {
  return choose_decode_w(ceil_pow2(ceil_pow2(m) + k), shard_bytes, max_nv);
}

KernelChoice choose_decode_w(uint64_t W, uint64_t shard_bytes, int max_nv) {
  if (W <= 32) {
    const int w = static_cast<int>(W);
    const int nv = clamp_nv(fit_nv(std::min(env_nv(4), max_nv), shard_bytes), w, false);
    return {Variant::kRegister, w, nv, reg_name(false, w, nv)};
  }
  return {Variant::kGeneric, static_cast<int>(W), 1, "decode_generic_nv1"};
}

KernelChoice choose_encode_low(uint64_t C, uint64_t shard_bytes, int max_nv) {
  static const char *kNames[6][3] = {
      {"encode_low_reg_w1_nv1", "encode_low_reg_w1_nv2", "encode_low_reg_w1_nv4"},
      {"encode_low_reg_w2_nv1", "encode_low_reg_w2_nv2", "encode_low_reg_w2_nv4"},
      {"encode_low_reg_w4_nv1", "encode_low_reg_w4_nv2", "encode_low_reg_w4_nv4"},
      {"encode_low_reg_w8_nv1", "encode_low_reg_w8_nv2", "encode_low_reg_w8_nv4"},
      {"encode_low_reg_w16_nv1", "encode_low_reg_w16_nv2", "encode_low_reg_w16_nv4"},
      {"encode_low_reg_w32_nv1", "encode_low_reg_w32_nv2", "encode_low_reg_w32_nv4"}};
  if (C <= 32) {  // coefficients + one recovery chunk live: the encode register budget
    const int c = static_cast<int>(C);
    const int nv = clamp_nv(fit_nv(std::min(env_nv(4), max_nv), shard_bytes), c, true);
    int si = 0;
    while ((1 << si) < c) si++;
    return {Variant::kRegister, c, nv, kNames[si][nv == 1 ? 0 : nv == 2 ? 1 : 2]};
  }
  return {Variant::kGeneric, static_cast<int>(C), 1, "encode_low_generic_nv1"};
}

#define RS_ENC_LOW_CASE(C_, NV_)                                                  \
  if (kc.size == C_ && kc.nv == NV_) {                                            \
    hipLaunchKernelGGL((k_encode_low_reg<C_, NV_>), grid, dim3(kBlock), 0, s, b); \
    e = hipGetLastError();                                                        \
    if (e != hipSuccess) return e;                                                \
    continue;                                                                     \
  }

static hipError_t launch_encode_low_phases(const EncodeArgs &a, hipStream_t s);

hipError_t launch_encode_low(const KernelChoice &kc, const EncodeArgs &a, hipStream_t s) {
  trace_launch(kc.name);
  // phase launches for every generic low-rate encode since the phase kernels stopped spilling
  // (round 5: RS(300,1000) 1 MiB x 16 33.1 -> 23.4 ms, 64 KiB x 8 1.25 -> 0.76 ms, RS(1000,4000)
  // 4 KiB x 64 2.74 -> 1.47 ms; profiles/r05/lowrate/encph.log). Round 4 kept the per-lane column
  // walk where it had enough waves (then 32.7 vs 41.7 ms at 1 MiB x 16).
  const char *ph = std::getenv("RS_AMD_LOW_ENC_PHASES");  // 1 / 0: force the phase launches / the walk
  const bool phases = ph && *ph ? std::strcmp(ph, "1") == 0 : true;
  if (kc.variant == Variant::kGeneric && a.chunk >= 64 && phases) return launch_encode_low_phases(a, s);
  if (kc.variant == Variant::kGeneric) {
    // a.scratch: `regions` C-position regions per stripe (low_encode): the coefficients, then
    // one per recovery chunk of a launch; the chunks run in groups of regions - 1
    const dim3 g = grid_for(a.shard_bytes, 1, a.n_stripes);
    hipLaunchKernelGGL(k_encode_low_coef<1>, g, dim3(kBlock), 0, s, a);
    if (hipError_t e = hipGetLastError()) return e;
    const uint32_t G = a.regions ? a.regions - 1 : a.n_chunks;
    if (G == 0 || G > 65535) return hipErrorInvalidValue;
    for (uint32_t j0 = 0; j0 < a.n_chunks; j0 += G) {
      EncodeArgs b = a;
      b.chunk0 = j0;
      hipLaunchKernelGGL(k_encode_low_generic<1>, dim3(g.x, g.y, std::min(G, a.n_chunks - j0)), dim3(kBlock), 0, s, b);
      if (hipError_t e = hipGetLastError()) return e;
    }
    return hipSuccess;
  }
  for (uint64_t s0 = 0; s0 < a.n_stripes; s0 += 65535) {
    EncodeArgs b = a;
    b.data += s0 * a.data_stripe_stride;
    b.parity += s0 * a.parity_stripe_stride;
    b.n_stripes = std::min<uint64_t>(65535, a.n_stripes - s0);
    const dim3 grid = grid_for(b.shard_bytes, kc.nv, b.n_stripes);
    hipError_t e = hipSuccess;
    RS_ENC_LOW_CASE(1, 1) RS_ENC_LOW_CASE(1, 2) RS_ENC_LOW_CASE(1, 4)
    RS_ENC_LOW_CASE(2, 1) RS_ENC_LOW_CASE(2, 2) RS_ENC_LOW_CASE(2, 4)
    RS_ENC_LOW_CASE(4, 1) RS_ENC_LOW_CASE(4, 2) RS_ENC_LOW_CASE(4, 4)
    RS_ENC_LOW_CASE(8, 1) RS_ENC_LOW_CASE(8, 2)
    RS_ENC_LOW_CASE(16, 1)
    RS_ENC_LOW_CASE(32, 1)
    return hipErrorInvalidValue;
  }
  return hipSuccess;
}
#undef RS_ENC_LOW_CASE

KernelChoice choose_decode_matrix(uint32_t n_out, uint64_t shard_bytes, int max_nv) {
  static const char *kNames[9][3] = {
      {"", "", ""},
      {"decode_matrix_e1_nv1", "decode_matrix_e1_nv2", "decode_matrix_e1_nv4"},
      {"decode_matrix_e2_nv1", "decode_matrix_e2_nv2", "decode_matrix_e2_nv4"},
      {"decode_matrix_e3_nv1", "decode_matrix_e3_nv2", "decode_matrix_e3_nv4"},
      {"decode_matrix_e4_nv1", "decode_matrix_e4_nv2", "decode_matrix_e4_nv4"},
      {"decode_matrix_e5_nv1", "decode_matrix_e5_nv2", "decode_matrix_e5_nv4"},
      {"decode_matrix_e6_nv1", "decode_matrix_e6_nv2", "decode_matrix_e6_nv4"},
      {"decode_matrix_e7_nv1", "decode_matrix_e7_nv2", "decode_matrix_e7_nv4"},
      {"decode_matrix_e8_nv1", "decode_matrix_e8_nv2", "decode_matrix_e8_nv4"}};
  const int nv = fit_nv(std::min(env_nv(4), max_nv), shard_bytes);
  const int ni = nv == 1 ? 0 : nv == 2 ? 1 : 2;
  KernelChoice kc{Variant::kMatrix, static_cast<int>(n_out), nv, kNames[n_out][ni]};
  kc.prefetch = 1;  // inputs in flight per lane (2 measured no faster)
  return kc;
}

KernelChoice choose_decode_mtile(uint32_t n_out, uint64_t shard_bytes, int max_nv) {
  (void)n_out;
  int nv = std::min(std::min(env_nv(1), max_nv), 2);
  if (shard_bytes % (512ull * nv)) nv = 1;
  return {Variant::kMatrixTiled, kMtileEW, nv, nv == 1 ? "decode_mtile16_nv1" : "decode_mtile16_nv2"};
}

#define RS_MAT_CASE(E_, NV_)                                                                  \
  if (kc.size == E_ && kc.nv == NV_) {                                                        \
    switch (kc.prefetch) {                                                                    \
      case 2: hipLaunchKernelGGL((k_decode_matrix<E_, NV_, 2>), grid, dim3(kBlock), 0, s, a); break; \
      default: hipLaunchKernelGGL((k_decode_matrix<E_, NV_, 1>), grid, dim3(kBlock), 0, s, a); break; \
    }                                                                                         \
    return hipGetLastError();                                                                 \
  }
#define RS_MAT_NV(E_) RS_MAT_CASE(E_, 1) RS_MAT_CASE(E_, 2) RS_MAT_CASE(E_, 4)

#define RS_ENC_CASE(C_, NV_)                                                  \
  if (kc.size == C_ && kc.nv == NV_) {                                        \
    hipLaunchKernelGGL((k_encode_reg<C_, NV_>), grid, dim3(kBlock), 0, s, a); \
    return hipGetLastError();                                                 \
  }
#define RS_DEC_CASE(W_, NV_)                                                  \
  if (kc.size == W_ && kc.nv == NV_) {                                        \
    hipLaunchKernelGGL((k_decode_reg<W_, NV_>), grid, dim3(kBlock), 0, s, a); \
    return hipGetLastError();                                                 \
  }

static hipError_t launch_encode_one(const KernelChoice &kc, const EncodeArgs &a, hipStream_t s);
static hipError_t launch_decode_one(const KernelChoice &kc, const DecodeArgs &a, hipStream_t s);

// The fused kernels map one stripe to one blockIdx.y (no stripe loop inside the
// kernel: a loop lets the compiler hoist every per-stripe-invariant uniform value
// into SGPRs and spill them), so batches are launched in slices of <= 65535 stripes.
hipError_t launch_encode(const KernelChoice &kc, const EncodeArgs &a, hipStream_t s) {
  trace_launch(kc.name);
  if (kc.variant == Variant::kGeneric) return launch_encode_one(kc, a, s);
  for (uint64_t s0 = 0; s0 < a.n_stripes; s0 += 65535) {
    EncodeArgs b = a;
    b.data += s0 * a.data_stripe_stride;
    b.parity += s0 * a.parity_stripe_stride;
    b.n_stripes = std::min<uint64_t>(65535, a.n_stripes - s0);
    hipError_t e = launch_encode_one(kc, b, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_decode(const KernelChoice &kc, const DecodeArgs &a, hipStream_t s) {
  trace_launch(kc.name);
  if (kc.variant == Variant::kGeneric) return launch_decode_one(kc, a, s);
  for (uint64_t s0 = 0; s0 < a.n_stripes; s0 += 65535) {
    DecodeArgs b = a;
    b.orig += s0 * a.orig_stripe_stride;
    b.rec += s0 * a.rec_stripe_stride;
    b.out += s0 * a.out_stripe_stride;
    if (b.xsrc) b.xsrc += s0 * a.xsrc_stripe_stride;
    b.tab_mat += s0 * a.mat_stride;
    b.pos_src += s0 * a.src_stride;
    if (b.nout) b.nout += s0;
    b.tab_pre += s0 * a.pattern_stride;
    b.tab_post += s0 * a.pattern_stride;
    b.pos_src += s0 * a.pattern_stride;
    b.pos_dst += s0 * a.pattern_stride;
    b.n_stripes = std::min<uint64_t>(65535, a.n_stripes - s0);
    hipError_t e = launch_decode_one(kc, b, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

static hipError_t launch_encode_one(const KernelChoice &kc, const EncodeArgs &a, hipStream_t s) {
  const dim3 grid = grid_for(a.shard_bytes, kc.nv, a.n_stripes);
  if (kc.variant == Variant::kRegister) {
    // live slots 2*C: NV <= 128 / (4*C)
    RS_ENC_CASE(1, 1) RS_ENC_CASE(1, 2) RS_ENC_CASE(1, 4)
    RS_ENC_CASE(2, 1) RS_ENC_CASE(2, 2) RS_ENC_CASE(2, 4)
    RS_ENC_CASE(4, 1) RS_ENC_CASE(4, 2) RS_ENC_CASE(4, 4)
    RS_ENC_CASE(8, 1) RS_ENC_CASE(8, 2)
    RS_ENC_CASE(16, 1)
    RS_ENC_CASE(32, 1)
    return hipErrorInvalidValue;
  }
  if (kc.variant == Variant::kWaveSplit) {
    // one block per 64-lane region; 4 waves split the 64 positions
    const uint64_t regions = a.shard_bytes / 64 * (8 / kc.nv) / 64;
    const dim3 g(static_cast<uint32_t>(regions), grid.y, 1);
    // LDS-staged VGPR tables (no SGPR->VGPR moves, no SGPR spills): RS(200,55) 256 KiB x 256
    // NV=1 7.36 vs 7.62 ms, NV=2 9.34 vs 11.5 ms against SGPR tables
    // (profiles/r01/sweep_rs200_55_ws64_lds.jsonl)
    if (kc.nv == 1) hipLaunchKernelGGL((k_encode_ws64l<1>), g, dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL((k_encode_ws64l<2>), g, dim3(kBlock), 0, s, a);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_encode_generic<1>, grid, dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

// the phases of xform_ph (same grouping): size N, lowest distance 2^dlo_log, first table
void xform_phases(uint64_t size, bool inv, std::vector<XPhase> &out) {
  uint32_t lg = 0;
  while ((1ull << lg) < size) lg++;
  const uint32_t n4 = lg / 2;
  uint32_t layer = 0;
  bool r2_done = !(lg & 1);
  uint64_t ti = 0;
  out.clear();
  do {
    const uint32_t c = std::min<uint32_t>(3, n4 - layer);
    const bool with_r2 = !r2_done && layer + c == n4 && c < 3;
    const uint32_t nn = (1u << (2 * c)) << (with_r2 ? 1 : 0);
    out.push_back({nn, inv ? 2 * layer : (with_r2 || c == 0 ? 0 : lg - 2 * (layer + c)), ti});
    for (uint32_t l = layer; l < layer + c; l++) ti += inv ? 3 * (size >> (2 * l + 2)) : 3ull << (2 * l);
    layer += c;
    r2_done = r2_done || with_r2 || c == 0;
  } while (layer < n4 || !r2_done);
}

static uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

// positions of the FFT's A and B buffers: those the phases after the first read (0 for one phase)
static uint64_t decode_y_rows(uint64_t W, uint64_t rmax_fft) {
  std::vector<XPhase> ph;
  xform_phases(W, false, ph);
  return ph.size() > 1 ? std::min(W, round_up(rmax_fft, 1ull << ph[0].dlo_log)) : 0;
}

// X (A written over it in place) | B. The first FFT phase reads every position of its
// sub-problem from X before it writes that sub-problem's A rows, and sub-problems are disjoint,
// so A needs no buffer of its own (X | A | B took ~3W rows per stripe at W = 65536)
uint64_t decode_generic_rows(uint64_t W, uint64_t trunc, uint64_t trunc_fft) {
  return W + decode_y_rows(W, trunc_fft ? trunc_fft : trunc);
}

// NS: the sub-problem sizes a mode runs with for W = 64 .. 65536 (xform_phases): the first
// phases and the middle ones are 64 points, only the last phases vary (instantiating just
// those keeps the build time down)
template <bool INV, int MODE, int NS>
static hipError_t launch_dphase(uint32_t n, dim3 g, const DecodeArgs &a, const PhaseArgs &q, hipStream_t s) {
  switch (n) {
#define RS_DPH_CASE(N_)                                                              \
  case N_:                                                                           \
    if constexpr ((NS & N_) != 0) {                                                  \
      hipLaunchKernelGGL((k_dphase<N_, INV, MODE>), g, dim3(kBlock), 0, s, a, q);    \
      break;                                                                         \
    } else {                                                                         \
      return hipErrorInvalidValue;                                                   \
    }
    RS_DPH_CASE(2) RS_DPH_CASE(4) RS_DPH_CASE(8) RS_DPH_CASE(16) RS_DPH_CASE(32) RS_DPH_CASE(64)
#undef RS_DPH_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// the first FFT phase with the IFFT's last phase fused in (64-point sub-problems)
static hipError_t launch_dphase_fused(uint32_t ni, dim3 g, const DecodeArgs &a, const PhaseArgs &q, hipStream_t s) {
  constexpr int M = kPhDeriv | kPhSplitB;
  switch (ni) {
#define RS_DPF_CASE(NI_) \
  case NI_: hipLaunchKernelGGL((k_dphase<64, false, M, NI_>), g, dim3(kBlock), 0, s, a, q); break;
    RS_DPF_CASE(2) RS_DPF_CASE(4) RS_DPF_CASE(8) RS_DPF_CASE(16) RS_DPF_CASE(32) RS_DPF_CASE(64)
#undef RS_DPF_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Decoder.decode (root.zig:268-335) over any W as one launch per transform phase
// (a.scratch: decode_generic_rows positions per stripe)
static hipError_t launch_decode_generic(const DecodeArgs &a, hipStream_t s) {
  const uint64_t W = a.work, sb = a.shard_bytes;
  if (W < 2 || (W & (W - 1)) || W > 65536 || sb % 64) return hipErrorInvalidValue;
  const uint64_t ri = std::min<uint64_t>(a.trunc, W), rf = std::min<uint64_t>(a.trunc_fft ? a.trunc_fft : a.trunc, W);
  const uint64_t ylen = decode_y_rows(W, rf), stride = (W + ylen) * sb;
  uint8_t *X = a.scratch, *Y = X, *B = X + W * sb;  // A in place over X (decode_generic_rows)
  const bool contig = contig_ok(sb, 1);
  const dim3 g0 = grid_for(sb, 1, 1);
  const uint32_t gz = static_cast<uint32_t>(std::min<uint64_t>(a.n_stripes, 65535));
  std::vector<XPhase> ph, iph;
  xform_phases(W, true, iph);
  // with two or more IFFT phases the last one runs inside the first FFT phase's loads (its
  // sub-problems are the union of G of the IFFT phase's): one pass over X less, and X read
  // before it is the previous phase's output
  const bool fuse = iph.size() >= 2;
  const size_t n_ifft = fuse ? iph.size() - 1 : iph.size();
  uint64_t lim = 0;  // positions the previous IFFT phase wrote (the rest are zero)
  for (size_t i = 0; i < n_ifft; i++) {
    ph.assign(1, iph[i]);
    const uint64_t span = static_cast<uint64_t>(ph[0].n) << ph[0].dlo_log, wl = round_up(ri, span);
    PhaseArgs q{X, X, stride, stride, i == 0 ? ri : lim, wl, sb, W, ri, ph[0].ti, a.tab_ifft, ph[0].dlo_log, nullptr,
                nullptr, contig, nullptr, 0, 0, 0};
    const dim3 g(g0.x, static_cast<uint32_t>(wl / ph[0].n), gz);
    hipError_t e = i == 0 ? launch_dphase<true, kPhGather, 64>(ph[0].n, g, a, q, s)
                          : launch_dphase<true, 0, 64>(ph[0].n, g, a, q, s);
    if (e != hipSuccess) return e;
    lim = wl;
  }
  xform_phases(W, false, ph);
  for (size_t i = 0; i < ph.size(); i++) {
    const uint64_t span = static_cast<uint64_t>(ph[i].n) << ph[i].dlo_log, wl = round_up(rf, span);
    const bool first = i == 0, last = i + 1 == ph.size();
    PhaseArgs q{first ? X : Y, Y, stride, stride, first ? (fuse ? lim : W) : ylen, ylen, sb, W, rf, ph[i].ti, a.tab_fft,
                ph[i].dlo_log, B, B, contig, a.tab_ifft, iph.back().ti, ri, iph.back().dlo_log};
    const dim3 g(g0.x, static_cast<uint32_t>(wl / ph[i].n), gz);
    if (first && fuse && (ph[i].n != 64 || last || (64u >> (iph.back().dlo_log - ph[i].dlo_log)) != iph.back().n))
      return hipErrorInvalidValue;  // the shapes xform_phases gives every W >= 128
    // first: W = 64 (one phase each way) or fused with the IFFT's last phase (W >= 128)
    hipError_t e = first && last ? launch_dphase<false, kPhDeriv | kPhScatter, 64>(ph[i].n, g, a, q, s)
                   : first       ? (fuse ? launch_dphase_fused(iph.back().n, g, a, q, s) : hipErrorInvalidValue)
                   : i == 1      ? (last ? launch_dphase<false, kPhLsum | kPhScatter, 126>(ph[i].n, g, a, q, s)
                                         : launch_dphase<false, kPhLsum, 64>(ph[i].n, g, a, q, s))
                   : last        ? launch_dphase<false, kPhScatter, 30>(ph[i].n, g, a, q, s)
                                 : hipErrorInvalidValue;  // no fourth FFT phase below W = 2^19
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <int MODE, int NS>
static hipError_t launch_ephase(uint32_t n, uint32_t ni, dim3 g, const EncodeArgs &a, const PhaseArgs &q, uint32_t subs,
                                uint32_t fc, hipStream_t s) {
  if (ni) {  // the first FFT phase with the IFFT's last phase: 64-point sub-problems
    if constexpr (MODE == kEpFft) {  // (never also the last phase, never an IFFT phase)
      if (n != 64) return hipErrorInvalidValue;
      switch (ni) {
#define RS_EPF_CASE(NI_) \
  case NI_: hipLaunchKernelGGL((k_ephase<64, MODE, NI_>), g, dim3(kBlock), 0, s, a, q, subs, fc); break;
        RS_EPF_CASE(2) RS_EPF_CASE(4) RS_EPF_CASE(8) RS_EPF_CASE(16) RS_EPF_CASE(32) RS_EPF_CASE(64)
#undef RS_EPF_CASE
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    } else {
      return hipErrorInvalidValue;
    }
  }
  switch (n) {
#define RS_EPH_CASE(N_)                                                                \
  case N_:                                                                             \
    if constexpr ((NS & N_) != 0) {                                                    \
      hipLaunchKernelGGL((k_ephase<N_, MODE, 0>), g, dim3(kBlock), 0, s, a, q, subs, fc); \
      break;                                                                           \
    } else {                                                                           \
      return hipErrorInvalidValue;                                                     \
    }
    RS_EPH_CASE(2) RS_EPH_CASE(4) RS_EPH_CASE(8) RS_EPH_CASE(16) RS_EPH_CASE(32) RS_EPH_CASE(64)
#undef RS_EPH_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// rs_gf.hpp scalar_encode_low as phase launches (k_ephase); a.scratch: a.regions C-row
// regions per stripe (coefficients + one per recovery chunk of a launch), chunk groups of
// regions - 1 as launch_encode_low's generic path
static hipError_t launch_encode_low_phases(const EncodeArgs &a, hipStream_t s) {
  const uint64_t C = a.chunk, sb = a.shard_bytes, k = a.k;
  if (C < 64 || (C & (C - 1)) || sb % 64) return hipErrorInvalidValue;
  const uint32_t R = a.regions ? a.regions : 1 + a.n_chunks, G = R - 1;
  if (G == 0) return hipErrorInvalidValue;
  const uint64_t stride = static_cast<uint64_t>(R) * C * sb;
  const bool contig = contig_ok(sb, 1);
  const dim3 g0 = grid_for(sb, 1, 1);
  const uint32_t gz = static_cast<uint32_t>(std::min<uint64_t>(a.n_stripes, 65535));
  const uint64_t ri = std::min<uint64_t>(k, C);
  std::vector<XPhase> iph, fph;
  xform_phases(C, true, iph);
  xform_phases(C, false, fph);
  const bool fuse = iph.size() >= 2;
  uint8_t *X = a.scratch;
  uint64_t lim = 0;
  for (size_t i = 0; i + (fuse ? 1 : 0) < iph.size(); i++) {
    const uint64_t span = static_cast<uint64_t>(iph[i].n) << iph[i].dlo_log, wl = round_up(ri, span);
    PhaseArgs q{X, X, stride, stride, i == 0 ? ri : lim, wl, sb, C, ri, iph[i].ti, a.tabs, iph[i].dlo_log, nullptr,
                nullptr, contig, nullptr, 0, 0, 0};
    const dim3 g(g0.x, static_cast<uint32_t>(wl / iph[i].n), gz);
    hipError_t e = i == 0 ? launch_ephase<kEpGather, 64>(iph[i].n, 0, g, a, q, 0, 0, s)
                          : launch_ephase<0, 64>(iph[i].n, 0, g, a, q, 0, 0, s);
    if (e != hipSuccess) return e;
    lim = wl;
  }
  const uint64_t TI = ifft_tab_count(C);
  for (uint32_t j0 = 0; j0 < a.n_chunks; j0 += G) {
    EncodeArgs b = a;
    b.chunk0 = j0;
    const uint32_t nc = std::min(G, a.n_chunks - j0);
    for (size_t i = 0; i < fph.size(); i++) {
      const bool first = i == 0, last = i + 1 == fph.size();
      const uint32_t subs = static_cast<uint32_t>(C / fph[i].n);
      if (static_cast<uint64_t>(subs) * nc > 65535) return hipErrorInvalidValue;
      // first: reads region 0 (the coefficients, with the IFFT's last phase fused in when
      // there is one); the others read their chunk's region
      PhaseArgs q{X, X, stride, stride, first ? (fuse ? lim : C) : C, 0, sb, C, 0, fph[i].ti, a.tabs + TI,
                  fph[i].dlo_log, nullptr, nullptr, contig, a.tabs, fuse ? iph.back().ti : 0, ri,
                  fuse ? iph.back().dlo_log : 0};
      const uint32_t ni = first && fuse ? iph.back().n : 0;
      if (ni && (fph[i].n != 64 || (64u >> (iph.back().dlo_log - fph[i].dlo_log)) != ni)) return hipErrorInvalidValue;
      const dim3 g(g0.x, subs * nc, gz);
      const uint32_t fc = first ? 0u : 1u;
      hipError_t e = last ? launch_ephase<kEpFft | kEpOut, 126>(fph[i].n, ni, g, b, q, subs, fc, s)
                          : launch_ephase<kEpFft, 64>(fph[i].n, ni, g, b, q, subs, fc, s);
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

// per stripe: coefficients (C) | block K's transform (C) | A' and B' (the final FFT's first-phase
// rows the later phases read)
static uint64_t low_block_ylen(uint64_t C, uint64_t k) {
  std::vector<XPhase> fph;
  xform_phases(C, false, fph);
  return round_up(k, 1ull << fph[0].dlo_log);
}
// the derivative applied whole (k_ephase DLO + k_lbfin1) where the IFFT has two phases
static bool low_block_whole(uint64_t C) {
  std::vector<XPhase> iph, fph;
  xform_phases(C, true, iph);
  xform_phases(C, false, fph);
  return iph.size() == 2 && fph.size() == 2 && iph[0].n == 64 && iph[0].dlo_log == 0;
}
// per stripe: X (coefficients) | R1 (block K's transform) | then W (its (I + D_lo) copy) | A'
// for the whole derivative, A' | B' for the split one
uint64_t low_block_rows(uint64_t C, uint64_t k) {
  return low_block_whole(C) ? 3 * C + low_block_ylen(C, k) : 2 * C + 2 * low_block_ylen(C, k);
}

static hipError_t launch_lbfin1(uint32_t ni, dim3 g, uint64_t n, const PhaseArgs &q, uint32_t u, uint32_t acc,
                                hipStream_t s) {
  switch (ni) {
#define RS_LB1_CASE(NI_) \
  case NI_: hipLaunchKernelGGL((k_lbfin1<NI_>), g, dim3(kBlock), 0, s, n, q, u, acc); break;
    RS_LB1_CASE(2) RS_LB1_CASE(4) RS_LB1_CASE(8) RS_LB1_CASE(16) RS_LB1_CASE(32) RS_LB1_CASE(64)
#undef RS_LB1_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

static hipError_t launch_lbfinal(uint32_t ni, dim3 g, uint64_t n, const PhaseArgs &q, const RsTab *gamma, uint32_t u,
                                 uint32_t acc, hipStream_t s) {
  switch (ni) {
#define RS_LBF_CASE(NI_) \
  case NI_:                                                                                   \
    if (u || !acc) hipLaunchKernelGGL((k_lbfinal<NI_, 0>), g, dim3(kBlock), 0, s, n, q, gamma, u, acc); \
    hipLaunchKernelGGL((k_lbfinal<NI_, 1>), g, dim3(kBlock), 0, s, n, q, gamma, u, acc);               \
    break;
    RS_LBF_CASE(2) RS_LBF_CASE(4) RS_LBF_CASE(8) RS_LBF_CASE(16) RS_LBF_CASE(32) RS_LBF_CASE(64)
#undef RS_LBF_CASE
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// rs_lowrate.cpp's block form as phase launches (scalar_reconstruct_low_blocks step by step):
//  1. coefficients of d' = IFFT_C(originals, erased ones zero, trunc k): its phases but the last
//     (k_ephase GATHER with a.skip), region 0;
//  2. per block K = j + 1 holding rows used: FFT_{C, skew KC}(coefficients) (the IFFT's last
//     phase fused into its first, as launch_encode_low_phases), its last phase forming the
//     syndromes (SYN) into region 1; the IFFT_{C, skew KC} of those, in place, but its last
//     phase, which runs inside k_lbfinal (the final FFT's first phase, accumulating A', B');
//  3. the final FFT's later phases: LSUM (A' + L B', D_C's low bits) and SCATTER (the erased
//     originals times exp(-L_g)) as launch_decode_generic's.
hipError_t launch_low_blocks(const LowBlockArgs &L, hipStream_t s) {
  const EncodeArgs &a = L.enc;
  const uint64_t C = a.chunk, sb = a.shard_bytes, k = a.k, mp = a.m;
  if (C < 128 || (C & (C - 1)) || C > 32768 || sb % 64 || k == 0 || k > C || mp == 0 || a.n_chunks == 0 ||
      mp > static_cast<uint64_t>(a.n_chunks) * C)
    return hipErrorInvalidValue;
  std::vector<XPhase> iph, fph;
  xform_phases(C, true, iph);
  xform_phases(C, false, fph);
  if (iph.size() < 2 || fph.size() < 2 || fph.size() > 3 || fph[0].n != 64 ||
      (64u >> (iph.back().dlo_log - fph[0].dlo_log)) != iph.back().n || (64ull << fph[0].dlo_log) != C)
    return hipErrorInvalidValue;  // the shapes xform_phases gives every C in [128, 32768]
  trace_launch("low_blocks");
  const uint64_t ylen = low_block_ylen(C, k), stride = low_block_rows(C, k) * sb;
  // two IFFT phases (C <= 4096): the derivative whole before the final FFT (k_ephase DLO +
  // k_lbfin1), so the final FFT's second phase is plain; else the A' / B' split (k_lbfinal, LSUM)
  const bool whole = low_block_whole(C);
  uint8_t *X = a.scratch, *R1 = X + C * sb, *Wr = whole ? X + 2 * C * sb : nullptr;
  uint8_t *Ap = X + (whole ? 3 : 2) * C * sb, *Bp = whole ? nullptr : Ap + ylen * sb;
  const bool contig = contig_ok(sb, 1);
  const dim3 g0 = grid_for(sb, 1, 1);
  const uint32_t gz = static_cast<uint32_t>(std::min<uint64_t>(a.n_stripes, 65535));
  const uint64_t TI = ifft_tab_count(C);
  uint64_t lim = 0;
  for (size_t i = 0; i + 1 < iph.size(); i++) {  // 1.
    const uint64_t span = static_cast<uint64_t>(iph[i].n) << iph[i].dlo_log, wl = round_up(k, span);
    PhaseArgs q{X, X, stride, stride, i == 0 ? k : lim, wl, sb, C, k, iph[i].ti, a.tabs, iph[i].dlo_log, nullptr,
                nullptr, contig, nullptr, 0, 0, 0};
    const dim3 g(g0.x, static_cast<uint32_t>(wl / iph[i].n), gz);
    hipError_t e = i == 0 ? launch_ephase<kEpGather, 64>(iph[i].n, 0, g, a, q, 0, 0, s)
                          : launch_ephase<0, 64>(iph[i].n, 0, g, a, q, 0, 0, s);
    if (e != hipSuccess) return e;
    lim = wl;
  }
  // 2. only the blocks holding a row used: an empty block's syndromes are zero and so is its
  // contribution (linear), so the first block run stores A' (B') and later ones accumulate
  bool stored = false;
  for (uint32_t j = 0; j < a.n_chunks; j++) {
    if (L.used && !L.used[j]) continue;
    EncodeArgs b = a;
    b.chunk0 = j;
    const uint64_t rj = std::min<uint64_t>(C, mp - static_cast<uint64_t>(j) * C);
    for (size_t i = 0; i < fph.size(); i++) {
      const bool first = i == 0, last = i + 1 == fph.size();
      const uint32_t subs = static_cast<uint32_t>(C / fph[i].n);
      PhaseArgs q{X, X, stride, stride, first ? lim : C, 0, sb, C, 0, fph[i].ti, a.tabs + TI, fph[i].dlo_log, nullptr,
                  nullptr, contig, a.tabs, iph.back().ti, k, iph.back().dlo_log};
      q.rec = L.rec;
      q.rec_stride = L.rec_stripe_stride;
      q.syn_idx = L.syn_idx;
      q.syn_tab = L.syn_tab;
      const dim3 g(g0.x, subs, gz);
      hipError_t e = last ? launch_ephase<kEpFft | kEpSyn, 126>(fph[i].n, 0, g, b, q, subs, 1, s)
                          : launch_ephase<kEpFft, 64>(fph[i].n, first ? iph.back().n : 0, g, b, q, subs, first ? 0 : 1, s);
      if (e != hipSuccess) return e;
    }
    uint64_t lj = rj;  // rows of region 1 the next phase reads (the rest are zero)
    const RsTab *ti = L.tabs_i + static_cast<uint64_t>(j) * TI;
    for (size_t i = 0; i + 1 < iph.size(); i++) {
      const uint64_t span = static_cast<uint64_t>(iph[i].n) << iph[i].dlo_log, wl = round_up(rj, span);
      PhaseArgs q{R1, R1, stride, stride, lj, wl, sb, C, rj, iph[i].ti, ti, iph[i].dlo_log, nullptr, whole ? Wr : nullptr,
                  contig, nullptr, 0, 0, 0};
      q.syn_tab = L.gamma1 + j;  // DLO: 1 + gamma of block K
      const dim3 g(g0.x, static_cast<uint32_t>(wl / iph[i].n), gz);
      hipError_t e = whole ? launch_ephase<kEpDlo, 64>(iph[i].n, 0, g, b, q, 0, 0, s)
                           : launch_ephase<0, 64>(iph[i].n, 0, g, b, q, 0, 0, s);
      if (e != hipSuccess) return e;
      lj = wl;
    }
    PhaseArgs q{R1, Ap, stride, stride, lj, ylen, sb, C, k, fph[0].ti, L.dec.tab_fft, fph[0].dlo_log, whole ? Wr : nullptr,
                Bp, contig, ti, iph.back().ti, rj, iph.back().dlo_log};
    const dim3 g(g0.x, static_cast<uint32_t>(C / 64), gz);
    hipError_t e = whole ? launch_lbfin1(iph.back().n, g, a.n_stripes, q, L.u[j], stored ? 1u : 0u, s)
                         : launch_lbfinal(iph.back().n, g, a.n_stripes, q, L.gamma + j, L.u[j], stored ? 1u : 0u, s);
    if (e != hipSuccess) return e;
    stored = true;
  }
  if (!stored) return hipErrorInvalidValue;  // no row used: the plan never asks for the block form
  DecodeArgs d = L.dec;  // 3.
  d.n_stripes = a.n_stripes;
  d.pattern_stride = 0;
  for (size_t i = 1; i < fph.size(); i++) {
    const bool last = i + 1 == fph.size();
    const uint64_t span = static_cast<uint64_t>(fph[i].n) << fph[i].dlo_log, wl = round_up(k, span);
    PhaseArgs q{Ap, Ap, stride, stride, ylen, ylen, sb, C, k, fph[i].ti, L.dec.tab_fft, fph[i].dlo_log, Bp, Bp, contig,
                nullptr, 0, 0, 0};
    const dim3 g(g0.x, static_cast<uint32_t>(wl / fph[i].n), gz);
    hipError_t e = whole  ? launch_dphase<false, kPhScatter, 126>(fph[i].n, g, d, q, s)
                   : i == 1 ? (last ? launch_dphase<false, kPhLsum | kPhScatter, 126>(fph[i].n, g, d, q, s)
                                    : launch_dphase<false, kPhLsum, 64>(fph[i].n, g, d, q, s))
                            : launch_dphase<false, kPhScatter, 30>(fph[i].n, g, d, q, s);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

static hipError_t launch_decode_one(const KernelChoice &kc, const DecodeArgs &a, hipStream_t s) {
  const dim3 grid = grid_for(a.shard_bytes, kc.nv, a.n_stripes);
  if (kc.variant == Variant::kRegister) {
    // live slots W: NV <= 128 / (2*W)
    RS_DEC_CASE(2, 1) RS_DEC_CASE(2, 2) RS_DEC_CASE(2, 4)
    RS_DEC_CASE(4, 1) RS_DEC_CASE(4, 2) RS_DEC_CASE(4, 4)
    RS_DEC_CASE(8, 1) RS_DEC_CASE(8, 2) RS_DEC_CASE(8, 4)
    RS_DEC_CASE(16, 1) RS_DEC_CASE(16, 2) RS_DEC_CASE(16, 4)
    RS_DEC_CASE(32, 1) RS_DEC_CASE(32, 2)
    return hipErrorInvalidValue;
  }
  if (kc.variant == Variant::kMatrixTiled) {
    const uint64_t regions = a.shard_bytes / 64 * (8 / kc.nv) / 64;
    const dim3 g(static_cast<uint32_t>(regions), grid.y, 1);
    // LDS-staged VGPR tables: -13 % against SGPR tables at NV=1
    if (kc.nv == 1) hipLaunchKernelGGL((k_decode_mtile_lds<kMtileEW, 1>), g, dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL((k_decode_mtile_lds<kMtileEW, 2>), g, dim3(kBlock), 0, s, a);
    return hipGetLastError();
  }
  if (kc.variant == Variant::kMatrix) {
    RS_MAT_NV(1) RS_MAT_NV(2) RS_MAT_NV(3) RS_MAT_NV(4)
    RS_MAT_NV(5) RS_MAT_NV(6) RS_MAT_NV(7) RS_MAT_NV(8)
    return hipErrorInvalidValue;
  }
  return launch_decode_generic(a, s);
}

hipError_t launch_pattern_plan(const uint8_t *d_present, uint64_t present_stride, uint32_t k, uint32_t m, uint32_t C,
                               uint32_t W, uint64_t n, uint32_t max_e, bool d1, bool low, const uint16_t *d_exp,
                               const uint16_t *d_log, const uint16_t *d_log_walsh, uint16_t *logs, RsTab *pre,
                               RsTab *post, int32_t *src, int32_t *dst, int32_t *status, hipStream_t s) {
  return launch_pattern_plan_impl(d_present, present_stride, k, m, C, W, n, max_e, d1, low, d_exp, d_log, d_log_walsh,
                                  logs, pre, post, src, dst, status, s);
}

hipError_t launch_pattern_matrix(const uint8_t *d_present, uint64_t present_stride, uint32_t k, uint32_t m, uint32_t C,
                                 uint32_t W, uint64_t n, uint32_t max_e, const uint16_t *logs, const RsTab *tab_ifft,
                                 const RsTab *tab_fft, const uint16_t *d_exp, const uint16_t *d_log, uint16_t *images,
                                 RsTab *tabs, int32_t *srcs, int32_t *nout, hipStream_t s) {
  return launch_pattern_matrix_impl(d_present, present_stride, k, m, C, W, n, max_e, logs, tab_ifft, tab_fft, d_exp,
                                    d_log, images, tabs, srcs, nout, s);
}

hipError_t launch_psyn_plan(const uint8_t *present, uint64_t present_stride, uint32_t k, uint32_t m, uint32_t max_out,
                            uint32_t max_e, uint64_t n, const uint16_t *G, const uint16_t *d_exp, const uint16_t *d_log,
                            uint32_t *plan, uint32_t plan_dw, int32_t *status, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (k > 256 || m > kPsynMaxM || max_out > m || plan_dw < (k + 31) / 32 + 2 + m * max_out) return hipErrorInvalidValue;
  trace_launch("k_psyn_plan");
  hipLaunchKernelGGL(k_psyn_plan, dim3(static_cast<uint32_t>((n + 63) / 64)), dim3(64), 0, s, present, present_stride,
                     k, m, max_out, max_e, n, G, d_exp, d_log, plan, plan_dw, status);
  return hipGetLastError();
}

uint32_t wps_coef_stride(uint32_t max_e) {
  return max_e <= kWpsMaxOut ? kWpsMaxOut : std::min(kWpsMaxM, (max_e + 7u) / 8u * 8u);
}

hipError_t launch_wps_plan(const uint8_t *present, uint64_t present_stride, uint32_t k, uint32_t m, uint32_t max_e,
                           uint64_t n, const uint16_t *G, const uint16_t *d_exp, const uint16_t *d_log, uint32_t *plan,
                           uint32_t plan_dw, uint32_t dmw, int32_t *status, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t cs = wps_coef_stride(max_e);
  if (m > kWpsMaxM || dmw < 2 || plan_dw < dmw + 2 + kWpsMaxM + kWpsMaxM * cs || (dmw - 2) * 32 < k)
    return hipErrorInvalidValue;
  trace_launch(cs == kWpsMaxOut ? "k_wps_plan" : "k_wps_plan_wave");
  if (cs == kWpsMaxOut) {
    hipLaunchKernelGGL(k_wps_plan, dim3(static_cast<uint32_t>((n + 63) / 64)), dim3(64), 0, s, present,
                       present_stride, k, m, max_e, n, G, d_exp, d_log, plan, plan_dw, dmw, status);
  } else {
    if (n > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_wps_plan_wave, dim3(static_cast<uint32_t>(n)), dim3(64), 0, s, present, present_stride, k, m,
                       max_e, G, d_exp, d_log, plan, plan_dw, dmw, cs, status);
  }
  return hipGetLastError();
}

// Per-stripe decode blocks of the fused FFT reconstruct (rs_fftnet.hpp decode_block, on
// the device): one thread per (stripe, slot). Slot 0 writes the mask words, the block
// mask, the rows R (the trimmed present rows), the output rows and the status; slot
// 1 + p the masks of L_p (recovery row p in R); slot 1 + m + g those of
// L'_g * beta_K (erased data shard g); unused slots write zero masks.
__device__ uint32_t to_uv_d(uint32_t x, const FdecConsts &c) {
  uint32_t lo = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) lo ^= (x >> (8 + i) & 1) ? c.p[i] : 0u;
  return x ^ lo;
}
__global__ __launch_bounds__(256) void k_fdec_block(const uint8_t *__restrict__ trimmed, uint32_t k, uint32_t m,
                                                    uint32_t C, uint32_t W, uint64_t n, uint32_t max_e,
                                                    const uint16_t *__restrict__ logs, const uint16_t *__restrict__ exp,
                                                    const uint16_t *__restrict__ log, uint32_t dwm, uint32_t mko,
                                                    uint32_t words, uint32_t *__restrict__ blk, int32_t *status,
                                                    FdecConsts cst) {
  const uint64_t slots = 1ull + m + k, gi = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (gi >= n * slots) return;
  const uint64_t s = gi / slots;
  const uint32_t slot = static_cast<uint32_t>(gi % slots);
  const uint8_t *pr = trimmed + s * (k + m);
  uint32_t *b = blk + s * words;
  const uint16_t *lg = logs + s * W;
  if (slot == 0) {
    uint32_t e = 0, used = 0;
    for (uint32_t g = 0; g < k; g++) e += pr[g] ? 0u : 1u;
    for (uint32_t p = 0; p < m; p++) used += pr[k + p] ? 1u : 0u;
    if (status) status[s] = used < e ? 2 : (e > max_e ? 14 : 0);  // NotEnoughShards / InvalidArgument
    for (uint32_t i = 0; i < mko; i++) b[i] = 0;
    for (uint32_t g = 0; g < k; g++) b[dwm + 3 + g] = 0xFFFFFFFFu;
    if (used < e) return;  // nothing restored
    uint32_t row = 0;  // more than max_e erased: the first max_e are restored (status 14)
    for (uint32_t g = 0; g < k; g++)
      if (!pr[g]) {
        b[g / 32] |= 1u << (g % 32);
        if (row < max_e) {
          b[dwm + 3 + g] = row++;
          b[dwm] |= 1u << ((C + g) / C);
        }
      }
    for (uint32_t p = 0; p < m; p++)
      if (pr[k + p]) b[dwm + 1 + p / 32] |= 1u << (p % 32);
    return;
  }
  uint32_t c = 0;
  if (slot <= m) {
    const uint32_t p = slot - 1;
    if (pr[k + p]) c = exp[lg[p]];  // root.zig:292-295
  } else {
    const uint32_t g = slot - 1 - m;
    if (!pr[g]) c = mul16_d(cst.beta[(C + g) / C], 65535u - lg[C + g], exp, log);  // root.zig:321-326
  }
  uint32_t *M = b + mko + 128u * (slot - 1);
  uint32_t cu[8], cv[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    cu[j] = c ? to_uv_d(mul16_d(to_uv_d(1u << j, cst), log[c], exp, log), cst) : 0u;
    cv[j] = c ? to_uv_d(mul16_d(to_uv_d(1u << (8 + j), cst), log[c], exp, log), cst) : 0u;
  }
  for (int i = 0; i < 8; i++)
    for (int j = 0; j < 8; j++) {
      M[16 * i + j] = ((cu[j] >> i & 1) ? 0x0F0F0F0Fu : 0u) | ((cv[j] >> (8 + i) & 1) ? 0xF0F0F0F0u : 0u);
      M[16 * i + 8 + j] = ((cv[j] >> i & 1) ? 0x0F0F0F0Fu : 0u) | ((cu[j] >> (8 + i) & 1) ? 0xF0F0F0F0u : 0u);
    }
}

hipError_t launch_fdec_plan(const uint8_t *present, uint64_t present_stride, uint32_t k, uint32_t m, uint32_t C,
                            uint32_t W, uint64_t n, uint32_t max_e, const uint16_t *d_exp, const uint16_t *d_log,
                            const uint16_t *d_log_walsh, uint8_t *trimmed, uint16_t *logs, uint32_t *blk,
                            uint32_t dwm, uint32_t mko, uint32_t words, const FdecConsts &cst, int32_t *status,
                            hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (W / C > 32 || mko < dwm + 3 + k || words < mko + 128 * (m + k)) return hipErrorInvalidValue;
  trace_launch("k_trim_present");
  trace_launch("k_erasure_logs");
  trace_launch("k_fdec_block");
  hipLaunchKernelGGL(k_trim_present, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0, s, present,
                     present_stride, k, m, n, trimmed);
  hipError_t e = hipGetLastError();
  for (uint64_t s0 = 0; e == hipSuccess && s0 < n; s0 += 65535) {
    const uint32_t cnt = static_cast<uint32_t>(std::min<uint64_t>(65535, n - s0));
    hipLaunchKernelGGL(k_erasure_logs, dim3(cnt), dim3(1024), 0, s, trimmed + s0 * (k + m), static_cast<uint64_t>(k + m),
                       k, m, C, W, 0u, d_log_walsh, d_log, logs + s0 * W);
    e = hipGetLastError();
  }
  if (e != hipSuccess) return e;
  const uint64_t threads = n * (1ull + m + k);
  hipLaunchKernelGGL(k_fdec_block, dim3(static_cast<uint32_t>((threads + 255) / 256)), dim3(256), 0, s, trimmed, k, m, C,
                     W, n, max_e, logs, d_exp, d_log, dwm, mko, words, blk, status, cst);
  return hipGetLastError();
}

hipError_t launch_trim_present(const uint8_t *present, uint64_t present_stride, uint32_t k, uint32_t m, uint64_t n,
                               uint8_t *out, hipStream_t s) {
  trace_launch("k_trim_present");
  hipLaunchKernelGGL(k_trim_present, dim3(static_cast<uint32_t>((n + 255) / 256)), dim3(256), 0, s, present,
                     present_stride, k, m, n, out);
  return hipGetLastError();
}

hipError_t launch_tail_pack(const uint8_t *src, uint64_t src_stripe_stride, uint8_t *dst, uint64_t dst_stripe_stride,
                            uint64_t sb, uint64_t n, bool unpack, hipStream_t s) {
  if (sb % 64 == 0 || n == 0) return hipSuccess;
  trace_launch("k_tail_pack");
  const uint64_t blocks = (n * 64 + 255) / 256;
  hipLaunchKernelGGL(k_tail_pack, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, src, src_stripe_stride, dst,
                     dst_stripe_stride, sb, n, unpack ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_engine_fft(uint8_t *work, uint64_t sb, uint64_t pos, uint64_t size, uint64_t trunc,
                             const RsTab *tabs, bool inverse, hipStream_t s) {
  const dim3 grid = grid_for(sb, 1, 1);
  trace_launch("k_engine_transform");
  hipLaunchKernelGGL(k_engine_transform, grid, dim3(kBlock), 0, s, work, sb, pos, size, trunc, tabs,
                     inverse ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_mul_scalar(uint8_t *chunks, uint64_t bytes, const RsTab *tab, hipStream_t s) {
  const dim3 grid = grid_for(bytes, 1, 1);
  trace_launch("k_mul_scalar");
  hipLaunchKernelGGL(k_mul_scalar, grid, dim3(kBlock), 0, s, chunks, bytes, tab);
  return hipGetLastError();
}

}  // namespace rs
