// rs_fftnet.hpp — bit-sliced additive-FFT encode kernels for wide codes
// (chunk = ceilPow2(m) of 32 or 64), generated per plan and compiled with hipRTC.
//
// The dense k -> m networks of rs_jit.hpp grow with k * m; the reference's
// Encoder.encode (root.zig:136-173) costs O(chunk log chunk) multiplies per chunk
// instead (RS(200,55): 785 per column against 11,000 for the dense map). These
// kernels run that FFT schedule (Generic.zig:15-147, group for group, truncation
// included) bit-sliced, with every twiddle a compile-time GF(2) network.
//
// Representation. A lane holds 16 symbols of a shard position
// as 8 dwords: dword i = bit-plane i of the "u" half (low nibble of every byte)
// and bit-plane i of the "v" half (high nibble), where x = u + beta_8 * v with
// u, v in the subfield GF(2^8) = span(beta_0..beta_7) of the Cantor basis
// (gf.zig:8-13; T: u = lo ^ P*hi, v = hi). Every twiddle of a position < 256 is
// in GF(2^8) (its log is a multiple of 257), and multiplication by a in GF(2^8)
// acts as the same 8x8 GF(2) matrix on u and on v: one 8-dword network per
// butterfly, half the work of a 16x16 map, and half the registers per symbol.
// Other twiddles (positions >= 256) use four 8x8 blocks and a nibble swap.
//
// Work split: a workgroup of chunk/8 waves covers a 2 KiB slice of every shard
// (64 lanes x 16 symbols); wave w holds 8 of the chunk's positions. Layers of
// bits 0..2 run in layout A (wave = high bits, code specialised per wave: their
// twiddles depend on the wave's bits), the others in layout B (wave = low bits,
// one code path for all waves); a transpose through LDS switches layouts. The
// XOR-fold accumulator of root.zig:150-166 lives in registers in layout B.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "rs_jit.hpp"

namespace rs {
namespace fftnet {

constexpr uint8_t kOutNone = 0;    // FFT output not stored
constexpr uint8_t kOutStore = 1;   // out[row] = parity row
constexpr uint8_t kOutXorRec = 2;  // out[row] = rec[row] ^ parity row (syndrome of a reconstruct)

struct Spec {
  uint32_t k = 0, m = 0;
  uint32_t flags = 0;             // RS_FLAG_QUIRK_D1 / D2 (encode schedule and multiply as the reference's)
  std::vector<uint8_t> skip;      // k entries (or empty): data shard read as zero (erased)
  std::vector<uint8_t> out_mode;  // m entries (or empty = all kOutStore)
  int prefetch = -1;              // next-chunk positions loaded early (-1: RS_AMD_FFT_PREFETCH, default 4)
  uint32_t pieces = 1;            // stripes per 2 KiB unit: 1, or 2 for 1 KiB shards (pieces())
  // the encode inverted (k == m == chunk): input = the m recovery shards, IFFT at skew 0,
  // FFT at skew chunk, output = the k originals (reconstruct with every original lost)
  bool inverse = false;
  // per-stripe masks (launch dmask): the data positions skipped and the rows stored
  // come from each stripe's mask block instead of skip / out_mode (one stripe per unit)
  bool dyn = false;
  // fused reconstruct (implies dyn, corrected multiply, no D2): the syndromes
  // s = rec ^ Enc(d') of the rows R, then the reference's erasure-locator decode
  // (root.zig:268-335) restricted to the residual codeword, which is zero on every
  // received data position: x_g = (L'_g beta_K) * FFT_{C, skew KC}(IFFT_{C, skew 0}(L_R s_R))
  // for erased g in data block K. The pattern is data (decode block).
  bool decode = false;
  // workgroup b walks units [b per, (b + 1) per) instead of b, b + grid, ...: one stripe's
  // units in a row (per-stripe decode blocks stay in the scalar cache)
  bool blocked = false;
  // fused reconstruct of ONE erasure pattern (decode without dyn; k + m flags): the pattern
  // compiled in — the locator scalars as constant multiplies, the rows R, the erased data
  // positions, the output rows and the blocks static, butterflies no erased shard needs
  // pruned. No decode block.
  std::vector<uint8_t> present;
};
// u32 words of a stripe's mask block (Spec::dyn): bit p of words [0, w - 2) = data shard
// p read as zero, bit q of the last 2 words = parity row q stored
uint32_t dyn_mask_words(const Spec &s);

// the inverse form exists for this code (single full chunk: k == m == chunk)
bool supports_inverse(uint64_t k, uint64_t m, uint64_t shard_bytes);

constexpr uint64_t kUnitBytes = 2048;  // shard bytes one workgroup covers per unit

// chunk 32 or 64, high rate, at most kMaxChunks IFFT chunks (code size), shards of
// whole 2 KiB units (or 1 KiB: a unit spans two stripes) with k * shard_bytes below
// 2 GiB (32-bit buffer offsets)
constexpr uint32_t kMaxChunks = 16;
bool supports(uint64_t k, uint64_t m, uint64_t shard_bytes, bool chunk16 = false);
uint32_t pieces(uint64_t shard_bytes);  // Spec::pieces for a shard size

std::string generate(const Spec &s, const std::string &name);
std::string cache_key(const Spec &s);
std::string kernel_name(const Spec &s);

// compiled kernel (cached per device and spec); async: background compile (see jit::get_source).
// A build whose registers spill to scratch is rebuilt with less prefetch (spills cost more
// than the prefetch gains). The wrong bytes of round 2's spilled builds were a store-data
// hazard, now closed for every build (profiles/r03/spill_root_cause.md, STB).
const jit::Kernel *get(const Spec &s, bool async, std::string &err, bool &pending);
bool compile_check(const Spec &s, std::string &err, double *ms, size_t *code_bytes);

// data [stripe][k][sb] (stride ds), rec [stripe][m][sb] (rs; read for kOutXorRec rows),
// out [stripe][m][sb] (os; only the rows out_mode stores are written)
// Spec::dyn: dmask = n_stripes blocks of dmask_words (or one block for every stripe:
// shared_mask, a batch with one erasure pattern)
hipError_t launch(const jit::Kernel &kn, const Spec &s, const uint8_t *data, uint64_t ds, const uint8_t *rec, uint64_t rs,
                  uint8_t *out, uint64_t os, uint64_t sb, uint64_t n_stripes, hipStream_t st,
                  const uint32_t *dmask = nullptr, uint32_t dmask_words = 0, bool shared_mask = false);

// ---- fused FFT reconstruct (Spec::decode). A pattern's decode block (u32 words):
//   [0, dmw)            dyn mask words: bit p = data shard p erased (read as zero)
//   [dmw]               bit K: data block K (positions [KC, KC + C)) has an erasure
//   [dmw + 1, dmw + 3)  bit p: recovery row p is one of the rows R used
//   [dmw + 3 + g]       output row of erased data shard g (0xFFFFFFFF: not erased)
//   [mko + 128 p]       runtime-multiply masks (scalar_masks) of L_p, p < m (0 off R)
//   [mko + 128 (m + g)] masks of L'_g * beta_K for erased g
uint32_t decode_block_words(const Spec &s);
uint32_t decode_mask_offset(const Spec &s);
// beta_K for the W / C blocks of the decode transform (W = ceilPow2(C + k)); false if
// the block structure does not reduce to one polynomial (it does for every code tried)
bool decode_betas(uint32_t k, uint32_t m, std::vector<uint16_t> &beta);
// the 128 nibble masks of multiplication by the element c in the kernel's (u|v) planes:
// out_i = XOR_j (x_j & M[16 i + j]) ^ (swap(x_j) & M[16 i + 8 + j])
void scalar_masks(uint16_t c, uint32_t *masks);
// T's constants p_i = beta_{8+i} + beta_8 beta_i (u = lo ^ sum hi_i p_i): the device plan
// kernel's (u|v) change of basis
void uv_basis(uint32_t p[8]);
// decode block of one erasure pattern (present: k + m flags) for e = #erased <= m;
// R = the first e present recovery rows. Returns RS_OK or an RS_ERR_* status.
int decode_block(const Spec &s, const uint8_t *present, uint32_t *blk);
// scalar check of the decode schedule (host): mismatching symbols over `trials`
// random stripes and patterns with e erasures
uint64_t decode_selftest(uint32_t k, uint32_t m, uint32_t e, int trials);

// Host check of the generator's arithmetic: runs the kernel's schedule with its
// T-coordinate matrices on scalar symbols and compares with scalar_encode.
// Returns the number of mismatching symbols over `trials` random inputs.
uint64_t selftest(const Spec &s, int trials);
// measurement builds (RS_AMD_FFT_DEBUG bit 6): copy the phase stamps (8 waves x 64 s_memtime
// values of workgroup 0's third unit) of the current device to host; 0 on success
int read_stamps(uint64_t *host, size_t n);

// Instruction estimate of the generated network ops (wave instructions per unit)
struct Stats {
  uint64_t ops_a = 0, ops_b = 0, ops_io = 0, subfield = 0, general = 0, xor_only = 0;
};
Stats stats(const Spec &s);

}  // namespace fftnet
}  // namespace rs
