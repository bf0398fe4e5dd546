// rs_lowlds.hip — low-rate codec kernels (§8 f4; the reference panics, parity unpinned) that
// keep a column's whole C-point transform state on chip: VGPRs across the waves of one
// workgroup, switched between layouts through LDS. Only the shards the codec reads and writes
// cross HBM. Built apart from rs_kernels.hip (which takes minutes).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "rs_device.hpp"
#include "rs_internal.hpp"
#include "rs_xform.hpp"

namespace rs {
namespace {

using dev::fft_sub;
using dev::ifft_sub;
using dev::opq;
using dev::row_rsrc;
using dev::Sym;
using dev::zero_rsrc;

// ---- The low-rate encode with a column's whole C-point state on chip (C = 512; VERDICT r5
// item 7). One 8-wave workgroup per (512-byte column, recovery chunk j, stripe): the 64 lanes of
// every wave are the 64 dword pairs of the column (the shard layout of the phase kernels) and the
// waves split the positions, 64 each in VGPRs, in one of two layouts:
//   P: wave w holds positions 64 w + q (q < 64): the IFFT's first phase (bits 0-5) and the FFT's
//      last phase (bits 0-2, eight 8-point sub-problems) run in it;
//   Q: wave w holds positions w + 8 t (t < 64): the IFFT's last phase (bits 6-8, fused as
//      ifft_last_in) and the FFT's first phase (bits 3-8) run in it.
// Twiddle tables stay wave-uniform in both (they depend on the bits a phase does not hold). The
// layouts switch through LDS in two rounds of 128 KiB (four target waves per round). Only the k
// originals are read and the chunk's recovery rows written: the coefficients are recomputed per
// chunk (one more IFFT per chunk against a C-row coefficient scratch written once and read per
// chunk). Phase kernels' traffic for RS(300,1000) 1 MiB x 16 was 3.4x algorithmic
// (profiles/r06/lowrate/traffic_summary_base.json).
typedef uint32_t u32x4l __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2l __attribute__((ext_vector_type(2)));
struct LowLdsTi {
  uint32_t ia, ib, fa, fb;  // first tables of the IFFT phases (64 @ bits 0-5, 8 @ bits 6-8) and FFT phases
  uint32_t n_ifft;          // ifft_tab_count(C): the chunks' FFT tables follow the IFFT's
};
// The layouts share one array of 64 registers. Each exchange runs in two rounds: in round R every
// wave sends the 32 positions of registers [32R, 32R + 32) (to all eight waves, four to each) and
// receives 32 into the same registers, so the Q layout is the P registers under the fixed
// permutation qreg: Q slot t (position w + 8t) lives in register 32 ((t >> 2) & 1) + 4 (t >> 3) + (t & 3).
// LDS entry (16 B per lane): the pair of positions a b128 moves, [target wave][source wave][pair].
// The end of a round: its LDS reads must complete before the barrier that lets the next round
// (or the next exchange) overwrite the buffer. Without the memory-clobbering wait the compiler
// sank a round's ds_reads below that barrier into the branch that used them, where other
// waves had already written the next exchange's data (k_rec_low_lds, round 6).
__device__ __forceinline__ void lds_reads_done_bar() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
}
__device__ __forceinline__ constexpr int qreg(int t) { return 32 * ((t >> 2) & 1) + 4 * (t >> 3) + (t & 3); }

template <int R>
__device__ __forceinline__ void lds_p_to_q(Sym<1> *r, u32x4l *x, uint32_t w, uint32_t lane) {
  // send: P slot q = c + 8 i (to wave c, its Q slot 8 w + i), i in [4R, 4R + 4), pairs i, i + 1
#pragma unroll
  for (int c = 0; c < 8; c++)
#pragma unroll
    for (int b = 0; b < 2; b++) {
      const Sym<1> &p0 = r[c + 8 * (4 * R + 2 * b)], &p1 = r[c + 8 * (4 * R + 2 * b + 1)];
      x[(c * 16 + w * 2 + b) * 64 + lane] = (u32x4l){p0.l[0], p0.h[0], p1.l[0], p1.h[0]};
    }
  __syncthreads();
  // receive: from wave src its slots t = 8 src + 4R + 2b, + 1
#pragma unroll
  for (int src = 0; src < 8; src++)
#pragma unroll
    for (int b = 0; b < 2; b++) {
      const u32x4l e = x[(w * 16 + src * 2 + b) * 64 + lane];
      Sym<1> &q0 = r[qreg(8 * src + 4 * R + 2 * b)], &q1 = r[qreg(8 * src + 4 * R + 2 * b + 1)];
      q0.l[0] = e.x;
      q0.h[0] = e.y;
      q1.l[0] = e.z;
      q1.h[0] = e.w;
    }
  lds_reads_done_bar();
}
template <int R>
__device__ __forceinline__ void lds_q_to_p(Sym<1> *r, u32x4l *x, uint32_t w, uint32_t lane) {
  // send: Q slot t (position w + 8t) to P wave t >> 3, its slot w + 8 (t & 7); t & 7 in [4R, 4R + 4)
#pragma unroll
  for (int T = 0; T < 8; T++)
#pragma unroll
    for (int b = 0; b < 2; b++) {
      const int t = 8 * T + 4 * R + 2 * b;
      const Sym<1> &p0 = r[qreg(t)], &p1 = r[qreg(t + 1)];
      x[(T * 16 + w * 2 + b) * 64 + lane] = (u32x4l){p0.l[0], p0.h[0], p1.l[0], p1.h[0]};
    }
  __syncthreads();
  // receive: from Q wave src its positions src + 8 (4R + 2b), + 8 = P slots q, q + 8
#pragma unroll
  for (int src = 0; src < 8; src++)
#pragma unroll
    for (int b = 0; b < 2; b++) {
      const u32x4l e = x[(w * 16 + src * 2 + b) * 64 + lane];
      Sym<1> &q0 = r[src + 8 * (4 * R + 2 * b)], &q1 = r[src + 8 * (4 * R + 2 * b + 1)];
      q0.l[0] = e.x;
      q0.h[0] = e.y;
      q1.l[0] = e.z;
      q1.h[0] = e.w;
    }
  lds_reads_done_bar();
}

// row offsets fit a 32-bit soffset (C * sb < 2^31: encode_low_lds_ok), so one buffer resource
// per stripe serves every row: a row's offset is a scalar computed where it is used, and the
// rows a wave does not have read through the zero-record resource (no traffic)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t stripe_rsrc(const uint8_t *base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(base), static_cast<short>(0), 0x7FFFFFFF, 0x00020000);
}

__global__ __launch_bounds__(512) void k_encode_low_lds(EncodeArgs a, LowLdsTi ti) {
  constexpr uint64_t C = 512;
  __shared__ u32x4l xch[128 * 64];  // 128 KiB: one exchange round
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
  const uint32_t sb = static_cast<uint32_t>(a.shard_bytes);
  const uint32_t io = dev::lane_byte_offset<1>(blockIdx.x, lane, true), io_h = io + 256u;
  const uint32_t j = blockIdx.y;  // recovery chunk
  const uint32_t ri = a.k < C ? a.k : static_cast<uint32_t>(C);
  const uint32_t rj = a.m - j * static_cast<uint32_t>(C) < C ? a.m - j * static_cast<uint32_t>(C) : static_cast<uint32_t>(C);
  for (uint64_t s = blockIdx.z; s < a.n_stripes; s += gridDim.z) {
    const RsTab *tabs = opq(a.tabs);
    const RsTab *tf = opq(a.tabs + ti.n_ifft + static_cast<uint64_t>(j) * a.tabs_per_chunk);
    // this wave's rows in P (positions 64 w + q < n_in read, the rest zero), opaque per stripe
    const uint32_t w64 = dev::opqu(64u * w);
    const uint32_t n_in = ri > w64 ? (ri - w64 < 64u ? ri - w64 : 64u) : 0u;
    Sym<1> v[64];
    const __amdgpu_buffer_rsrc_t rd = stripe_rsrc(a.data + s * a.data_stripe_stride), rz = zero_rsrc();
#pragma unroll
    for (int q = 0; q < 64; q++) {
      const uint32_t so = (w64 + q) * sb;
      const __amdgpu_buffer_rsrc_t r = static_cast<uint32_t>(q) < n_in ? rd : rz;
      v[q].l[0] = __builtin_amdgcn_raw_buffer_load_b32(r, io, so, 0);
      v[q].h[0] = __builtin_amdgcn_raw_buffer_load_b32(r, io_h, so, 0);
    }
#pragma unroll
    for (int q = 0; q < 64; q++) dev::pair_halves(v[q], true);
    if (n_in) ifft_sub<64, 1>(v, tabs, ti.ia, C, ri, w64, 0);  // bits 0-5 (a wave past the originals holds zeros)
    lds_p_to_q<0>(v, xch, w, lane);
    lds_p_to_q<1>(v, xch, w, lane);
    // Q: the IFFT's last phase on the eight 8-point groups (bits 6-8), then the FFT's first (bits 3-8)
    Sym<1> u[64];
#pragma unroll
    for (int t = 0; t < 64; t++) u[t] = v[qreg(t)];
#pragma unroll
    for (int g = 0; g < 8; g++) {
      Sym<1> gr[8];
#pragma unroll
      for (int t = 0; t < 8; t++) gr[t] = u[g + 8 * t];
      ifft_sub<8, 1>(gr, tabs, ti.ib, C, ri, 0, 6);
#pragma unroll
      for (int t = 0; t < 8; t++) u[g + 8 * t] = gr[t];
    }
    fft_sub<64, 1>(u, tf, ti.fa, C, rj, 0, 3);
#pragma unroll
    for (int t = 0; t < 64; t++) v[qreg(t)] = u[t];
    lds_q_to_p<0>(v, xch, w, lane);
    lds_q_to_p<1>(v, xch, w, lane);
    // P: the FFT's last phase (bits 0-2) and the chunk's recovery rows jC + p, p < rj
    const uint32_t w64b = dev::opqu(64u * w);
    const uint32_t n_out = rj > w64b ? (rj - w64b < 64u ? rj - w64b : 64u) : 0u;
    if (n_out) {
#pragma unroll
      for (int sg = 0; sg < 8; sg++) fft_sub<8, 1>(v + 8 * sg, tf, ti.fb, C, rj, w64b + 8 * sg, 0);
      const __amdgpu_buffer_rsrc_t rp =
          stripe_rsrc(a.parity + s * a.parity_stripe_stride + static_cast<uint64_t>(j) * C * sb);
#pragma unroll
      for (int q = 0; q < 64; q++) {
        dev::pair_halves(v[q], true);
        const uint32_t so = (w64b + q) * sb;
        const __amdgpu_buffer_rsrc_t r = static_cast<uint32_t>(q) < n_out ? rp : rz;
        __builtin_amdgcn_raw_buffer_store_b32(v[q].l[0], r, io, so, 0);
        __builtin_amdgcn_raw_buffer_store_b32(v[q].h[0], r, io_h, so, 0);
      }
    }
  }
}

// ---- The low-rate reconstruct in block form with the state on chip (C = 512, the rows read all in
// one block K = j + 1; launch_low_blocks' scratch sequence otherwise). Same workgroup, layouts and
// exchanges as k_encode_low_lds; per (column, stripe), every step of launch_low_blocks in VGPRs:
//  1. d' (the received originals, the erased ones zero): IFFT_C (P: bits 0-5, Q: bits 6-8);
//  2. FFT_{C, skew KC} truncated at the block's last row read (Q: bits 3-8, P: bits 0-2) and the
//     syndromes s_r = (rec_r ^ Enc(d')_r) L_r sigma_K of the rows used (zero elsewhere) in P;
//  3. U = IFFT_{C, skew KC}(s) (P then Q);
//  4. Z = D_C U + gamma U for u = 1 (Z = U for u = 0): in Q a wave holds bits 3-8 of its
//     positions, so the derivative's terms over those are in its registers (ascending, in
//     place: a term reads positions above, still the original U); the terms over bits 0-2 are
//     another wave's same slot, read from LDS where every wave stored its original U first;
//  5. FFT_{C, skew 0} truncated at k (Q, then P) and the erased originals times g^(65535 - e_g)
//     stored to their output slots.
// HBM: the k - e received originals, the rows used and the e restored originals, once.
__global__ __launch_bounds__(512) void k_rec_low_lds(LowBlockArgs L, LowLdsTi ti, uint32_t j, uint32_t u) {
  constexpr uint64_t C = 512;
  __shared__ u32x4l xch[128 * 64];  // 128 KiB
  const EncodeArgs &a = L.enc;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
  const uint32_t sb = static_cast<uint32_t>(a.shard_bytes);
  const uint32_t io = dev::lane_byte_offset<1>(blockIdx.x, lane, true), io_h = io + 256u;
  const uint32_t k = a.k;
  const uint32_t rj = a.m - j * static_cast<uint32_t>(C) < C ? a.m - j * static_cast<uint32_t>(C) : static_cast<uint32_t>(C);
  typedef const __attribute__((address_space(4))) uint32_t *CU;
  typedef const __attribute__((address_space(4))) int32_t *CI;
  const __amdgpu_buffer_rsrc_t rz = zero_rsrc();
  for (uint64_t s = blockIdx.z; s < a.n_stripes; s += gridDim.z) {
    const uint32_t w64 = dev::opqu(64u * w);
    Sym<1> v[64];
    // 1. d' in P: received originals 64 w + q < k (the skip mask's two words of this wave)
    {
      const uint32_t n_in = k > w64 ? (k - w64 < 64u ? k - w64 : 64u) : 0u;
      const uint32_t nw = (k + 31u) >> 5, w0 = w64 >> 5;  // the mask's words (k bits)
      const uint64_t sk = n_in ? ((w0 + 1 < nw ? static_cast<uint64_t>(((CU)a.skip)[w0 + 1]) << 32 : 0ull) | ((CU)a.skip)[w0])
                               : ~0ull;
      const __amdgpu_buffer_rsrc_t rd = stripe_rsrc(a.data + s * a.data_stripe_stride);
#pragma unroll
      for (int q = 0; q < 64; q++) {
        const bool rdq = static_cast<uint32_t>(q) < n_in && !((sk >> q) & 1u);
        const __amdgpu_buffer_rsrc_t r = rdq ? rd : rz;
        const uint32_t so = (w64 + q) * sb;
        v[q].l[0] = __builtin_amdgcn_raw_buffer_load_b32(r, io, so, 0);
        v[q].h[0] = __builtin_amdgcn_raw_buffer_load_b32(r, io_h, so, 0);
      }
#pragma unroll
      for (int q = 0; q < 64; q++) dev::pair_halves(v[q], true);
      if (n_in) ifft_sub<64, 1>(v, opq(a.tabs), ti.ia, C, k, w64, 0);
    }
    lds_p_to_q<0>(v, xch, w, lane);
    lds_p_to_q<1>(v, xch, w, lane);
    {
      Sym<1> uq[64];
#pragma unroll
      for (int t = 0; t < 64; t++) uq[t] = v[qreg(t)];
#pragma unroll
      for (int g = 0; g < 8; g++) {  // the IFFT's last phase (bits 6-8)
        Sym<1> gr[8];
#pragma unroll
        for (int t = 0; t < 8; t++) gr[t] = uq[g + 8 * t];
        ifft_sub<8, 1>(gr, opq(a.tabs), ti.ib, C, k, 0, 6);
#pragma unroll
        for (int t = 0; t < 8; t++) uq[g + 8 * t] = gr[t];
      }
      // 2. FFT_{C, skew KC} of the coefficients, its first phase (bits 3-8)
      fft_sub<64, 1>(uq, opq(a.tabs + ti.n_ifft + static_cast<uint64_t>(j) * a.tabs_per_chunk), ti.fa, C, rj, 0, 3);
#pragma unroll
      for (int t = 0; t < 64; t++) v[qreg(t)] = uq[t];
    }
    lds_q_to_p<0>(v, xch, w, lane);
    lds_q_to_p<1>(v, xch, w, lane);
    const uint32_t n_s = rj > w64 ? (rj - w64 < 64u ? rj - w64 : 64u) : 0u;
    if (n_s) {  // wave-uniform: this wave holds rows of the block below its truncation
      const RsTab *tf = opq(a.tabs + ti.n_ifft + static_cast<uint64_t>(j) * a.tabs_per_chunk);
      const CI si = (CI)(L.syn_idx + static_cast<uint64_t>(j) * C + w64);
      const __amdgpu_buffer_rsrc_t rr = stripe_rsrc(L.rec + s * L.rec_stripe_stride + static_cast<uint64_t>(j) * C * sb);
      // the rows used, loaded one batch of 8 positions ahead of the syndromes that need them
      Sym<1> ta[8], tb[8];
      auto load8 = [&](int b0, Sym<1> *t) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
          const int q = b0 + i;
          const bool used = static_cast<uint32_t>(q) < n_s && si[q] >= 0;
          const __amdgpu_buffer_rsrc_t r = used ? rr : rz;
          const uint32_t so = (w64 + q) * sb;
          t[i].l[0] = __builtin_amdgcn_raw_buffer_load_b32(r, io, so, 0);
          t[i].h[0] = __builtin_amdgcn_raw_buffer_load_b32(r, io_h, so, 0);
        }
      };
      load8(0, ta);
#pragma unroll
      for (int sg = 0; sg < 8; sg++)  // the FFT's last phase (bits 0-2)
        fft_sub<8, 1>(v + 8 * sg, tf, ti.fb, C, rj, w64 + 8 * sg, 0);
#pragma unroll
      for (int b = 0; b < 8; b++) {
        Sym<1> *cur = (b & 1) ? tb : ta, *nxt = (b & 1) ? ta : tb;
        if (b + 1 < 8) load8(8 * (b + 1), nxt);
#pragma unroll
        for (int i = 0; i < 8; i++) {
          const int q = 8 * b + i;
          if (static_cast<uint32_t>(q) < n_s && si[q] >= 0) {  // wave-uniform
            dev::pair_halves(cur[i], true);
            dev::xor_into(v[q], cur[i]);
            dev::mul_inplace(v[q], dev::load_tab(opq(L.syn_tab) + static_cast<uint64_t>(j) * C + w64 + q));
          } else {
            dev::zero(v[q]);
          }
          dev::group_fence();
        }
      }
      // 3. U = IFFT_{C, skew KC}(s): its first phase (bits 0-5)
      ifft_sub<64, 1>(v, opq(L.tabs_i + static_cast<uint64_t>(j) * ti.n_ifft), ti.ia, C, rj, w64, 0);
    } else {
#pragma unroll
      for (int q = 0; q < 64; q++) dev::zero(v[q]);
    }
    lds_p_to_q<0>(v, xch, w, lane);
    lds_p_to_q<1>(v, xch, w, lane);
    {
      Sym<1> uq[64];
#pragma unroll
      for (int t = 0; t < 64; t++) uq[t] = v[qreg(t)];
#pragma unroll
      for (int g = 0; g < 8; g++) {  // its last phase (bits 6-8)
        Sym<1> gr[8];
#pragma unroll
        for (int t = 0; t < 8; t++) gr[t] = uq[g + 8 * t];
        ifft_sub<8, 1>(gr, opq(L.tabs_i + static_cast<uint64_t>(j) * ti.n_ifft), ti.ib, C, rj, 0, 6);
#pragma unroll
        for (int t = 0; t < 8; t++) uq[g + 8 * t] = gr[t];
      }
      // 4. Z = (1 + gamma) U + the derivative's neighbour terms (u = 1), in two halves of t
      if (u) {
        u32x2l *xu = reinterpret_cast<u32x2l *>(xch);
        const dev::Tab g1 = dev::load_tab(opq(L.gamma1) + j);
#pragma unroll
        for (int h = 0; h < 2; h++) {
#pragma unroll
          for (int t = 32 * h; t < 32 * h + 32; t++) xu[(w * 32 + (t - 32 * h)) * 64 + lane] = (u32x2l){uq[t].l[0], uq[t].h[0]};
          __syncthreads();
#pragma unroll
          for (int t = 32 * h; t < 32 * h + 32; t++) {  // ascending: the terms read positions above
            Sym<1> z = uq[t];
            dev::mul_inplace(z, g1);
#pragma unroll
            for (int x = 1; x < 64; x <<= 1)
              if (!(t & x)) dev::xor_into(z, uq[t + x]);
#pragma unroll
            for (uint32_t bb = 1; bb < 8; bb <<= 1) {  // the bit-0..2 neighbour: wave w | bb (none if set)
              const u32x2l e = xu[((w | bb) * 32 + (t - 32 * h)) * 64 + lane];
              const uint32_t keep = (w & bb) ? 0u : ~0u;  // wave-uniform, branch-free
              z.l[0] ^= e.x & keep;
              z.h[0] ^= e.y & keep;
            }
            uq[t] = z;
            dev::group_fence();
          }
          lds_reads_done_bar();
        }
      }
      // 5. the final FFT_{C, skew 0}, truncated at k: its first phase (bits 3-8)
      fft_sub<64, 1>(uq, opq(L.dec.tab_fft), ti.fa, C, k, 0, 3);
#pragma unroll
      for (int t = 0; t < 64; t++) v[qreg(t)] = uq[t];
    }
    lds_q_to_p<0>(v, xch, w, lane);
    lds_q_to_p<1>(v, xch, w, lane);
    const uint32_t n_o = k > w64 ? (k - w64 < 64u ? k - w64 : 64u) : 0u;
    if (n_o) {
#pragma unroll
      for (int sg = 0; sg < 8; sg++) fft_sub<8, 1>(v + 8 * sg, opq(L.dec.tab_fft), ti.fb, C, k, w64 + 8 * sg, 0);
      const CI dst = (CI)(L.dec.pos_dst + w64);
      const __amdgpu_buffer_rsrc_t ro = stripe_rsrc(L.dec.out + s * L.dec.out_stripe_stride);
#pragma unroll
      for (int q = 0; q < 64; q++) {
        const int32_t dq = static_cast<uint32_t>(q) < n_o ? dst[q] : -1;
        if (dq >= 0) {  // wave-uniform: an erased original, times g^(65535 - e_g)
          dev::mul_inplace(v[q], dev::load_tab(opq(L.dec.tab_post) + w64 + q));
          dev::pair_halves(v[q], true);
          const uint32_t so = static_cast<uint32_t>(dq) * sb;
          __builtin_amdgcn_raw_buffer_store_b32(v[q].l[0], ro, io, so, 0);
          __builtin_amdgcn_raw_buffer_store_b32(v[q].h[0], ro, io_h, so, 0);
        }
        dev::group_fence();
      }
    }
  }
}

}  // namespace

// the LDS-resident low-rate encode (k_encode_low_lds): C = 512, whole 512-byte columns;
// RS_AMD_LOW_LDS=0 keeps the phase launches
bool encode_low_lds_ok(uint64_t C, uint64_t sb) {
  const char *e = std::getenv("RS_AMD_LOW_LDS");
  if (e && std::strcmp(e, "0") == 0) return false;
  return C == 512 && sb % 512 == 0 && C * sb < (1ull << 31);  // row offsets in a 32-bit soffset
}

hipError_t launch_encode_low_lds(const EncodeArgs &a, hipStream_t s) {
  const uint64_t C = a.chunk, sb = a.shard_bytes;
  if (!encode_low_lds_ok(C, sb) || a.k == 0 || a.k > C || a.m == 0 || a.n_chunks == 0 ||
      static_cast<uint64_t>(a.n_chunks) * C < a.m || a.n_chunks > 65535 || !a.contig)
    return hipErrorInvalidValue;
  if (a.n_stripes == 0) return hipSuccess;
  std::vector<XPhase> iph, fph;
  xform_phases(C, true, iph);
  xform_phases(C, false, fph);
  if (iph.size() != 2 || fph.size() != 2 || iph[0].n != 64 || iph[0].dlo_log != 0 || iph[1].n != 8 ||
      iph[1].dlo_log != 6 || fph[0].n != 64 || fph[0].dlo_log != 3 || fph[1].n != 8 || fph[1].dlo_log != 0)
    return hipErrorInvalidValue;  // the layouts P / Q of the kernel
  trace_launch("encode_low_lds");
  const LowLdsTi ti{static_cast<uint32_t>(iph[0].ti), static_cast<uint32_t>(iph[1].ti),
                    static_cast<uint32_t>(fph[0].ti), static_cast<uint32_t>(fph[1].ti),
                    static_cast<uint32_t>(ifft_tab_count(C))};
  const dim3 g(static_cast<uint32_t>(sb / 512), a.n_chunks, static_cast<uint32_t>(std::min<uint64_t>(a.n_stripes, 65535)));
  hipLaunchKernelGGL(k_encode_low_lds, g, dim3(512), 0, s, a, ti);
  return hipGetLastError();
}


bool rec_low_lds_ok(uint64_t C, uint64_t sb) { return encode_low_lds_ok(C, sb); }

// one used block j (launch_low_blocks' sequence otherwise); u: the block's scalar form
hipError_t launch_rec_low_lds(const LowBlockArgs &L, uint32_t j, hipStream_t s) {
  const EncodeArgs &a = L.enc;
  const uint64_t C = a.chunk, sb = a.shard_bytes;
  if (!rec_low_lds_ok(C, sb) || a.k == 0 || a.k > C || a.m == 0 || j >= a.n_chunks || static_cast<uint64_t>(j) * C >= a.m ||
      !a.skip || !L.syn_idx || !L.syn_tab || !L.tabs_i || !L.gamma1 || !L.u || !L.dec.tab_fft || !L.dec.tab_post ||
      !L.dec.pos_dst)
    return hipErrorInvalidValue;
  if (a.n_stripes == 0) return hipSuccess;
  std::vector<XPhase> iph, fph;
  xform_phases(C, true, iph);
  xform_phases(C, false, fph);
  if (iph.size() != 2 || fph.size() != 2 || iph[0].n != 64 || iph[0].dlo_log != 0 || iph[1].n != 8 ||
      iph[1].dlo_log != 6 || fph[0].n != 64 || fph[0].dlo_log != 3 || fph[1].n != 8 || fph[1].dlo_log != 0)
    return hipErrorInvalidValue;
  trace_launch("reconstruct_low_lds");
  const LowLdsTi ti{static_cast<uint32_t>(iph[0].ti), static_cast<uint32_t>(iph[1].ti),
                    static_cast<uint32_t>(fph[0].ti), static_cast<uint32_t>(fph[1].ti),
                    static_cast<uint32_t>(ifft_tab_count(C))};
  const dim3 g(static_cast<uint32_t>(sb / 512), 1, static_cast<uint32_t>(std::min<uint64_t>(a.n_stripes, 65535)));
  hipLaunchKernelGGL(k_rec_low_lds, g, dim3(512), 0, s, L, ti, j, static_cast<uint32_t>(L.u[j]));
  return hipGetLastError();
}

}  // namespace rs
