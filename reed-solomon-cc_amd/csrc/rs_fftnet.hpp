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

// Host check of the generator's arithmetic: runs the kernel's schedule with its
// T-coordinate matrices on scalar symbols and compares with scalar_encode.
// Returns the number of mismatching symbols over `trials` random inputs.
uint64_t selftest(const Spec &s, int trials);

// Instruction estimate of the generated network ops (wave instructions per unit)
struct Stats {
  uint64_t ops_a = 0, ops_b = 0, ops_io = 0, subfield = 0, general = 0, xor_only = 0;
};
Stats stats(const Spec &s);

}  // namespace fftnet
}  // namespace rs
