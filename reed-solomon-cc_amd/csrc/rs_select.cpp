// rs_select.cpp — which kernel family a call runs on (networks, FFT kernels,
// syndrome path, table kernels) and the rs_*_kernel_name ABI that reports it.
#include "rs_host.hpp"

namespace rs {
namespace host {

// Encodes of 1 / 2 KiB shards stay on the table kernels, which measured as fast or
// faster there (RS(10,4) 2 KiB 0.644 vs 0.678 ms, RS(4,2) 1 KiB 0.528 vs 0.541 ms,
// profiles/r01/sweep_small_shard_networks.jsonl); reconstructs take the networks
// (RS(10,4) 1 KiB losing 4: 1.16 -> 0.67 ms). RS_AMD_NET_SMALL_ENCODE=1 overrides.
// Encode maps past the synchronous network cap that no FFT kernel covers run as
// background-compiled networks (table kernels until they land): with the shared-input
// form for several tiles and one tile otherwise, every shape measured is faster than the
// table register kernel — RS(40,12) 1 MiB 4.08 -> 2.95 ms, RS(100,6) 2.85 -> 2.35 ms,
// RS(100,4) 2.49 -> 2.30 ms, RS(200,8) 2.75 -> 2.58 ms (profiles/r02/sweep_encode_async_net.jsonl).
bool encode_net_async(uint64_t k, uint64_t m) {
  const char *sh = std::getenv("RS_AMD_NET_SHARED");
  if (sh && *sh && std::strcmp(sh, "0") == 0) return false;
  return m <= jit::kMaxOut && !fftnet::supports(k, m, fftnet::kUnitBytes) &&
         jit::supports_async(static_cast<uint32_t>(k), static_cast<uint32_t>(m), jit::kUnitBytes);
}

bool encode_net_ok(uint64_t sb) {
  if (jit::net_pieces(sb) == 1) return true;
  const char *e = std::getenv("RS_AMD_NET_SMALL_ENCODE");
  return e && *e && std::strcmp(e, "0") != 0;
}

// Multiplies the FFT reconstruct performs for a pattern (plan-time estimate used to
// choose between the FFT kernels and the matrix kernel).
uint64_t fft_decode_mul_count(uint64_t k, uint64_t m, uint64_t present_count, uint64_t e) {
  const uint64_t C = ceil_pow2(m), end = C + k, W = ceil_pow2(C + k);
  const uint16_t *sk = tables().skew;
  auto live = [&](uint64_t idx) -> uint64_t { return idx < kModulus && sk[idx] != kModulus ? 1 : 0; };
  auto group = [&](uint64_t r, uint64_t d) {  // m01 + m23 over d pairs, m02 over 2d
    const uint64_t b = r + d - 1;
    return d * (live(b) + live(b + 2 * d)) + 2 * d * live(b + d);
  };
  uint64_t n = present_count + e;  // erasure masks + reveal (root.zig:292-303, 321-326)
  uint64_t d = 1;                  // IFFT, Generic.zig:80-147
  for (uint64_t d4 = 4; d4 <= W; d = d4, d4 <<= 2)
    for (uint64_t r = 0; r < end; r += d4) n += group(r, d);
  if (d < W) n += d * live(d - 1);
  uint64_t d4 = W;  // FFT, Generic.zig:15-78
  for (uint64_t dd = W >> 2; dd != 0; d4 = dd, dd >>= 2)
    for (uint64_t r = 0; r < end; r += d4) n += group(r, dd);
  if (d4 == 2)
    for (uint64_t r = 0; r < end; r += 2) n += live(r);
  return n;
}

const char *decode_mode_env() {
  const char *e = std::getenv("RS_AMD_DECODE");
  return e ? e : "auto";
}


// Reconstruct kernel family for a pattern: 0 = FFT kernels (root.zig:268-335 as
// written), 1 = matrix (e <= 8, one wave), 2 = output-tiled matrix (e <= 64).
// The matrix kernels do k*e MACs at ~3/4 the cost of an FFT multiply (selectors
// shared across outputs); the FFT register kernels exist for W <= 32 only, beyond
// that the FFT path is the scratch-walking generic kernel (~10x slower per op).
int decode_kind(uint64_t k, uint64_t m, uint32_t flags, uint64_t e, uint64_t present_count, uint64_t sb) {
  (void)flags;
  const std::string mode = decode_mode_env();
  if (mode == "fft" || e == 0 || (k + m) > 4096) return 0;
  const uint64_t W = ceil_pow2(ceil_pow2(m) + k);
  const bool small_ok = e <= kMatrixMaxOut;
  const bool tiled_ok = e <= kMtileMaxOut && sb % 512 == 0;
  if (mode == "matrix") return small_ok ? 1 : tiled_ok ? 2 : 0;
  uint64_t fft_cost = 4 * fft_decode_mul_count(k, m, present_count, e);
  if (W > 32) fft_cost *= 10;  // generic kernel
  if (3 * k * e > fft_cost) return 0;
  return small_ok ? 1 : tiled_ok ? 2 : 0;
}

// Multiplies of one encode (root.zig:136-173) per 64-B column (live twiddles only).
uint64_t fft_encode_mul_count(uint64_t k, uint64_t m) {
  const uint64_t C = ceil_pow2(m);
  const uint16_t *sk = tables().skew;
  auto live = [&](uint64_t idx) -> uint64_t { return idx < kModulus && sk[idx] != kModulus ? 1 : 0; };
  auto group = [&](uint64_t b, uint64_t d) { return d * (live(b) + live(b + 2 * d)) + 2 * d * live(b + d); };
  const std::vector<uint64_t> truncs = encode_chunk_truncs(k, m, false);
  uint64_t n = 0;
  for (size_t j = 0; j < truncs.size(); j++) {  // IFFT per chunk, Generic.zig:80-147
    const uint64_t sd = (j + 1) * C;
    uint64_t d = 1;
    for (uint64_t d4 = 4; d4 <= C; d = d4, d4 <<= 2)
      for (uint64_t r = 0; r < truncs[j]; r += d4) n += group(r + d + sd - 1, d);
    if (d < C) n += d * live(d + sd - 1);
  }
  uint64_t d4 = C;  // FFT, Generic.zig:15-78
  for (uint64_t dd = C >> 2; dd != 0; d4 = dd, dd >>= 2)
    for (uint64_t r = 0; r < m; r += d4) n += group(r + dd - 1, dd);
  if (d4 == 2)
    for (uint64_t r = 0; r < m; r += 2) n += live(r);
  return n;
}

// a direct n_in -> e reconstruct map past the synchronous cap, within the background one
// A direct map past the synchronous cap, compiled in the background. For codes with an
// FFT kernel a large map loses to the syndrome path (FFT encode + e x e map): RS(200,55)
// losing 20 5.21 vs 3.90 ms, losing 14 3.56 vs 3.54, losing 8 2.61 vs 3.26 ms
// (profiles/r02/sweep_direct_vs_syndrome.jsonl), hence the n_in * e bound.
bool syndrome_pick(uint64_t k, uint64_t m, uint64_t e, uint32_t flags, uint64_t sb, const std::string &mode);
bool direct_net_async(uint64_t e, uint64_t n_in, uint64_t sb, const std::string &mode, uint64_t k, uint64_t m,
                      uint32_t flags) {
  if (mode == "auto" && fft_enabled() && fftnet::supports(k, m, sb) && n_in * e >= 2800 &&
      syndrome_pick(k, m, e, flags, sb, mode))
    return false;
  return (mode == "auto" || mode == "net") && jit::enabled() &&
         !jit::supports(static_cast<uint32_t>(n_in), static_cast<uint32_t>(e), sb) &&
         jit::supports_async(static_cast<uint32_t>(n_in), static_cast<uint32_t>(e), sb);
}

// Reconstruct by syndromes instead of the k x e matrix: worth it for wide codes
// with many erasures (RS(200,55) losing 55: 785 + 0.75*55^2 multiplies per column
// against 0.75*200*55). Needs the corrected multiply (under D1 the literal
// reconstruct is no inverse of the encode) and a fused (non-generic) encode kernel.
bool syndrome_pick(uint64_t k, uint64_t m, uint64_t e, uint32_t flags, uint64_t sb, const std::string &mode) {
  if (literal_decode(k, m, flags) || e == 0 || e > kMtileMaxOut || sb % 512) return false;
  if (choose_encode(k, m, sb, 4).variant == Variant::kGeneric) return false;
  if (mode == "syndrome") return true;
  if (mode != "auto") return false;
  const double direct = 0.75 * static_cast<double>(k) * e;
  const double syn = static_cast<double>(fft_encode_mul_count(k, m)) + 0.75 * static_cast<double>(e) * e;
  return syn < 0.7 * direct;
}

// Names of the kernels a call with 16-byte aligned buffers would run (bit-sliced
// networks: "net_<role>_i<inputs>_o<outputs>"; the hipRTC symbol rs_net_... adds a content hash).
const char *net_name(const char *role, uint64_t n_in, uint64_t n_out) {
  thread_local std::string name;
  name = std::string("net_") + role + "_i" + std::to_string(n_in) + "_o" + std::to_string(n_out);
  return name.c_str();
}

}  // namespace host
}  // namespace rs

using namespace rs;
using namespace rs::host;

extern "C" {

const char *rs_encode_kernel_name(uint64_t k, uint64_t m, size_t sb) {
  if (is_low_rate(k, m)) return low_encode_kernel_name(k, m, sb);
  if (fft_enabled() && fftnet::supports(k, m, sb)) return net_name("fft_encode", k, m);
  if (jit::enabled() && encode_net_ok(sb) &&
      (jit::supports(static_cast<uint32_t>(k), static_cast<uint32_t>(m), sb) ||
       (encode_net_async(k, m) && jit::supports_async(static_cast<uint32_t>(k), static_cast<uint32_t>(m), sb) &&
        jit::net_pieces(sb) == 1)))
    return net_name("encode", k, m);
  return choose_encode(k, m, sb, 4).name;
}
const char *rs_reconstruct_kernel_name(uint64_t k, uint64_t m, size_t sb, const uint8_t *present) {
  std::vector<uint8_t> def;
  if (!present) {
    def.assign(k + m, 1);
    for (uint64_t i = 0; i < std::min(k, m); i++) def[i] = 0;
    present = def.data();
  }
  uint64_t e = 0, have = 0;
  for (uint64_t i = 0; i < k; i++) e += present[i] ? 0 : 1;
  for (uint64_t i = 0; i < k + m; i++) have += present[i] ? 1 : 0;
  if (is_low_rate(k, m)) return low_reconstruct_kernel_name(k, m, sb, e);
  const std::string mode = decode_mode_env();
  if (e == k && have == m && (mode == "auto" || mode == "net") && fft_enabled() && fftnet::supports_inverse(k, m, sb))
    return net_name("fft_inverse", m, k);
  if ((mode == "auto" || mode == "net") && jit::enabled() &&
      jit::supports(static_cast<uint32_t>(k), static_cast<uint32_t>(e), sb))
    return net_name("reconstruct", k, e);
  // wide codes: the fused FFT reconstruct (every pattern's first calls; the steady state
  // unless a network beats it: a direct map for few losses, the syndrome e x e map for
  // e >= 3/4 m — rs_plans.cpp get_decode_plan)
  if (m <= 64 && fdec_mode() != 0 && fdec_supports(k, m, sb, flags_none()) && e > 0 && !(e == k && have == m) &&
      (mode == "auto" || mode == "net")) {
    const bool syn = syndrome_pick(k, m, e, flags_none(), sb, mode);
    const bool direct = decode_kind(k, m, flags_none(), e, have, sb) != 0 && direct_net_async(e, k, sb, mode, k, m, flags_none());
    if (!direct && k <= kPdecMaxK && pdec_enabled()) return net_name("fft_pdecode", k, m);  // steady state: the pattern compiled in
    if (fdec_mode() == 1 || !(direct || (syn && 4 * e >= 3 * m && jit::enabled() &&
                                         jit::supports_async(static_cast<uint32_t>(e), static_cast<uint32_t>(e), sb))))
      return net_name("fft_decode", k, m);
  }
  if (decode_kind(k, m, flags_none(), e, have, sb) != 0 && direct_net_async(e, k, sb, mode, k, m, flags_none()))
    return net_name("reconstruct", k, e);
  if (syndrome_pick(k, m, e, flags_none(), sb, mode)) {
    thread_local std::string name;
    name = std::string("syndrome+") +
           (fft_enabled() && fftnet::supports(k, m, sb) ? net_name("fft_encode", k, m) : choose_encode(k, m, sb, 4).name) +
           "+";
    if (jit::enabled() && jit::supports_async(static_cast<uint32_t>(e), static_cast<uint32_t>(e), sb))
      name += net_name("syndrome", e, e);
    else
      name += e <= kMatrixMaxOut ? choose_decode_matrix(static_cast<uint32_t>(e), sb, 4).name
                                 : choose_decode_mtile(static_cast<uint32_t>(e), sb, 4).name;
    return name.c_str();
  }
  switch (decode_kind(k, m, flags_none(), e, have, sb)) {
    case 1: return choose_decode_matrix(static_cast<uint32_t>(e), sb, 4).name;
    case 2: return choose_decode_mtile(static_cast<uint32_t>(e), sb, 4).name;
    default: return choose_decode(k, m, sb, 4).name;
  }
}

}  // extern "C"
