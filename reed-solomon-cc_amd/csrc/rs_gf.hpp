// rs_gf.hpp — GF(2^16) field tables and the per-multiplier v_perm tables (host side).
//
// Field: order 65536, polynomial 0x1002D, 16-element Cantor basis (gf.zig:1-13).
// Tables are generated once at library load, as tables.zig:22-147 does at build
// time: exp/log (22-45), LCH skew factors (60-87), log_walsh = FWHT(log) (146-147).
//
// Device multiply (rs_device.hpp) works on a GF(2)-linear decomposition of the
// 16-bit symbol x = lo | hi << 8 into six bit fields — lo[2:0], lo[5:3], lo[7:6],
// hi[2:0], hi[5:3], hi[7:6] — so each field indexes an <=8-entry byte table that
// one v_perm_b32 resolves for 4 symbols at once. RsTab holds, for one multiplier
// exp[log_m], those tables for the low and the high output byte. This replaces
// the reference's 4 x 16-entry nibble tables (mul_128, tables.zig:96-118) that
// x86 pshufb needs; both compute mul16(x, log_m) (utilities.zig:5-8) exactly.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace rs {

constexpr uint32_t kOrder = 65536;
constexpr uint32_t kModulus = 65535;
constexpr uint32_t kPolynomial = 65581;

// 96-byte table block for one multiplier (uniform across a wave; scalar-loaded).
// lo[]/hi[]: field tables for the low / high output byte, dword-packed:
//   [0,1] field lo[2:0] entries 0-3 | 4-7   [2,3] lo[5:3]   [4] lo[7:6]
//   [5,6] field hi[2:0]                     [7,8] hi[5:3]   [9] hi[7:6]
struct alignas(16) RsTab {
  uint32_t lo[10];
  uint32_t hi[10];
  uint32_t flags;  // bit 0: twiddle is log 65535 (element 0) -> XOR-only butterfly
  uint32_t log_m;
  uint32_t pad[2];
};
static_assert(sizeof(RsTab) == 96, "RsTab layout");

constexpr uint32_t kTabXorOnly = 1u;

struct Tables {
  uint16_t exp[kOrder];
  uint16_t log[kOrder];
  uint16_t skew[kModulus];
  uint16_t log_walsh[kOrder];
};

const Tables &tables();  // built once, thread-safe
// the Cantor basis (gf.zig:8-13) in polynomial form: a symbol v is the element
// XOR of cantor_basis()[i] over its set bits i (polynomial 0x1002D coordinates)
const uint16_t *cantor_basis();

inline uint16_t add_mod(uint32_t x, uint32_t y) {  // utilities.zig:10-13
  uint32_t s = x + y;
  return static_cast<uint16_t>(s + (s >> 16));
}
inline uint16_t sub_mod(uint32_t x, uint32_t y) {  // utilities.zig:15-18
  uint32_t d = x + kModulus - y;
  return static_cast<uint16_t>(d + (d >> 16));
}
uint16_t mul16(uint16_t x, uint16_t log_m);  // utilities.zig:5-8

// v_perm tables for an arbitrary GF(2)-linear map on 16-bit symbols, given the
// images of the 16 basis symbols 1 << b.
RsTab make_tab_from_images(const uint16_t images[16]);
// v_perm tables for multiplication by exp[log_m]; quirk_d1 reproduces
// Generic.zig:283 (hi product of nibble 0 read from t1_hi).
RsTab make_tab(uint16_t log_m, bool quirk_d1);
// The engine's multiply as a scalar map (Generic.zig:275-298, with D1 if asked).
uint16_t mul_engine(uint16_t x, uint16_t log_m, bool quirk_d1);

// ---- scalar (one symbol per position) restatement of the codec, used only to
// derive reconstruct matrices at plan time (host, per erasure pattern).
// Applies the reconstruct of root.zig:268-335 to W = ceilPow2(chunk+k) symbols:
// sym[pos] holds the received symbols (recovery at [0,m), originals at
// [chunk, chunk+k)); `received` flags positions; on return the missing
// originals hold their restored symbols. `erasures` = evalPoly output for the
// pattern (root.zig:277-289), computed once by the caller.
void scalar_reconstruct(uint16_t *sym, const uint8_t *received, const uint16_t *erasures, uint64_t k, uint64_t m,
                        bool quirk_d1);
// Encoder.encode (root.zig:136-173) on one symbol per shard: in[k] -> out[m]
// (used to derive the encode map for the bit-sliced network kernels).
void scalar_encode(const uint16_t *in, uint64_t k, uint64_t m, bool quirk_d1, bool quirk_d2, uint16_t *out);
// Low-rate encode (pow2(k) < pow2(m), or equal with k > m), on one symbol per shard.
// The reference has none (root.zig:119-121 @panic("TODO")); restated from the
// algorithm it ports, reed-solomon-simd's low-rate encoder (named in
// benchmarks.zig:1-2, not vendored: parity unpinned): originals at positions
// [0, k) of a chunk C = ceilPow2(k): IFFT(size C, trunc k, skew 0); recovery
// chunk j = FFT(copy, size C, trunc min(C, m - jC), skew (j+1)C).
void scalar_encode_low(const uint16_t *in, uint64_t k, uint64_t m, bool quirk_d1, uint16_t *out);
// Low-rate reconstruct (the decode the low-rate encode above implies; parity unpinned).
// The low-rate codeword is the evaluation of one polynomial P of degree < C on positions
// [0, C + m): originals at [0, k), known zeros at [k, C) (the encode's zero padding), recovery
// at [C, C + m). In a W = ceilPow2(C + m) point transform the positions [C + m, W) hold
// unknown values of P, so they join the erasures (missing originals, missing recovery);
// [k, C) stay received zeros. Then the formal-derivative decode of root.zig:268-335:
// evalPoly(W) -> received x g^e -> IFFT(W, trunc C + m) -> derivative -> FFT(W, trunc k) ->
// missing original i x g^(65535 - e_i). `received` has W entries in this position layout.
void erasure_logs_low(const uint8_t *received, uint64_t k, uint64_t m, uint16_t *out);
void scalar_reconstruct_low(uint16_t *sym, const uint8_t *received, const uint16_t *erasures, uint64_t k, uint64_t m);
// Generic.zig:80-147 / 15-78 on one symbol per position (pos 0, skew_delta sd, size points,
// groups r >= trunc skipped)
void scalar_ifft(uint16_t *s, uint64_t size, uint64_t trunc, uint64_t sd, bool quirk_d1);
void scalar_fft(uint16_t *s, uint64_t size, uint64_t trunc, uint64_t sd, bool quirk_d1);
// IFFT chunk truncations of the encode schedule (root.zig:143-166; D2 drops the last full chunk)
std::vector<uint64_t> encode_chunk_truncs(uint64_t k, uint64_t m, bool quirk_d2);
// root.zig:277-289: erasure flags for a received pattern -> evalPoly -> logs (65536 entries)
// (entries [0, ceilPow2(C + k)) are evaluated; the rest stay 0)
void erasure_logs(const uint8_t *received, uint64_t k, uint64_t m, uint16_t *out);
// test hook: erasure_logs* take eval_poly's two transforms even for small erased sets
void set_erasure_logs_fwht(bool on);
// Table for an FFT/IFFT twiddle: XOR-only marker when log_m == 65535
// (the engine's `log_m == gf.modulus` shortcut, Generic.zig:38,47,53,103,...).
RsTab make_twiddle(uint32_t skew_index, bool quirk_d1);

// walsh_hadamard.zig:16-62 (ones'-complement mod-65535 FWHT, truncated to m)
void fwht(uint16_t *data, uint64_t m);
// Generic.zig:200-215
void eval_poly(uint16_t *erasures, uint64_t truncated_size);

uint64_t ceil_pow2(uint64_t v);

// ---- butterfly schedules: the table sequence a device transform consumes.
// Mirrors Generic.zig:15-78 (fft) and 80-147 (ifft) group-for-group for ALL
// groups r < size; the device skips groups r >= truncated_size at run time.
size_t ifft_tab_count(uint64_t size);
size_t fft_tab_count(uint64_t size);
void push_ifft_tabs(std::vector<RsTab> &out, uint64_t size, uint64_t skew_delta, bool quirk_d1);
void push_fft_tabs(std::vector<RsTab> &out, uint64_t size, uint64_t skew_delta, bool quirk_d1);

}  // namespace rs
