// rs_gf.cpp — field tables, v_perm table builder, FWHT / evalPoly (host).
// See rs_gf.hpp for the reference citations.
#include "rs_gf.hpp"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

namespace rs {

namespace {

constexpr uint16_t kCantor[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                  0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};

std::unique_ptr<Tables> g_tables;
std::once_flag g_once;

uint16_t mul16_raw(uint16_t x, uint16_t lm, const uint16_t *exp, const uint16_t *log) {
  return x == 0 ? 0 : exp[add_mod(log[x], lm)];
}

void build(Tables &t) {
  // tables.zig:22-31 — LFSR over the polynomial; `exp` temporarily holds logs.
  std::memset(&t, 0, sizeof t);
  uint32_t state = 1;
  for (uint32_t i = 0; i < kModulus; i++) {
    t.exp[state] = static_cast<uint16_t>(i);
    state <<= 1;
    if (state >= kOrder) state ^= kPolynomial;
  }
  t.exp[0] = kModulus;
  // tables.zig:35-45 — re-express in the Cantor basis, invert.
  t.log[0] = 0;
  for (int i = 0; i < 16; i++) {
    uint32_t w = 1u << i;
    for (uint32_t j = 0; j < w; j++) t.log[j + w] = t.log[j] ^ kCantor[i];
  }
  for (uint32_t i = 0; i < kOrder; i++) t.log[i] = t.exp[t.log[i]];
  for (uint32_t i = 0; i < kOrder; i++) t.exp[t.log[i]] = static_cast<uint16_t>(i);
  t.exp[kModulus] = t.exp[0];

  // tables.zig:60-87 — LCH skew factors (as logs).
  uint16_t temp[15];
  for (int i = 1; i < 16; i++) temp[i - 1] = static_cast<uint16_t>(1u << i);
  for (int m = 0; m < 15; m++) {
    const uint32_t step = 1u << (m + 1);
    const uint32_t back = (1u << m) - 1;
    t.skew[back] = 0;
    for (int i = m; i < 15; i++) {
      const uint32_t s = 1u << (i + 1);
      for (uint32_t j = back; j < s; j += step) t.skew[j + s] = t.skew[j] ^ temp[i];
    }
    temp[m] = static_cast<uint16_t>(kModulus - t.log[mul16_raw(temp[m], t.log[temp[m] ^ 1], t.exp, t.log)]);
    for (int i = m + 1; i < 15; i++) temp[i] = mul16_raw(temp[i], add_mod(t.log[temp[i] ^ 1], temp[m]), t.exp, t.log);
  }
  for (uint32_t i = 0; i < kModulus; i++) t.skew[i] = t.log[t.skew[i]];

  // tables.zig:146-147
  std::memcpy(t.log_walsh, t.log, sizeof t.log);
  fwht(t.log_walsh, kOrder);
}

}  // namespace

const uint16_t *cantor_basis() { return kCantor; }

const Tables &tables() {
  std::call_once(g_once, [] {
    g_tables.reset(new Tables);
    build(*g_tables);
  });
  return *g_tables;
}

uint16_t mul16(uint16_t x, uint16_t log_m) {
  const Tables &t = tables();
  return mul16_raw(x, log_m, t.exp, t.log);
}

uint64_t ceil_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

uint16_t mul_engine(uint16_t x, uint16_t log_m, bool quirk_d1) {
  if (!quirk_d1) return mul16(x, log_m);
  // Generic.zig:283 (D1): prod_hi uses t1_hi[lo & 15], i.e. the hi byte of
  // mul(((lo & 15) << 4) ^ (x & 0xFFF0)) — still GF(2)-linear in x.
  const uint16_t xh = static_cast<uint16_t>(((x & 0xF) << 4) ^ (x & 0xFFF0));
  return static_cast<uint16_t>((mul16(x, log_m) & 0xFF) | (mul16(xh, log_m) & 0xFF00));
}

RsTab make_tab_from_images(const uint16_t images[16]) {
  // field f: bit offset in x and width; tables hold byte_o(map(v << off)).
  static constexpr int kOff[6] = {0, 3, 6, 8, 11, 14};
  static constexpr int kBits[6] = {3, 3, 2, 3, 3, 2};
  static constexpr int kSlot[6] = {0, 2, 4, 5, 7, 9};
  RsTab t{};
  for (int f = 0; f < 6; f++) {
    for (uint32_t v = 0; v < (1u << kBits[f]); v++) {
      uint16_t p = 0;
      for (int b = 0; b < kBits[f]; b++)
        if (v >> b & 1) p ^= images[kOff[f] + b];
      const int w = kSlot[f] + (v >> 2), sh = 8 * (v & 3);
      t.lo[w] |= static_cast<uint32_t>(p & 0xFF) << sh;
      t.hi[w] |= static_cast<uint32_t>(p >> 8) << sh;
    }
  }
  return t;
}

RsTab make_tab(uint16_t log_m, bool quirk_d1) {
  uint16_t img[16];
  for (int b = 0; b < 16; b++) img[b] = mul_engine(static_cast<uint16_t>(1u << b), log_m, quirk_d1);
  RsTab t = make_tab_from_images(img);
  t.flags = 0;
  t.log_m = log_m;
  return t;
}

namespace {
// scalar butterflies (Generic.zig:149-192) and transforms (15-147), pos = 0
inline void fft_bf_s(uint16_t &x, uint16_t &y, uint16_t lm, bool q) {
  if (lm != kModulus) x ^= mul_engine(y, lm, q);
  y ^= x;
}
inline void ifft_bf_s(uint16_t &x, uint16_t &y, uint16_t lm, bool q) {
  y ^= x;
  if (lm != kModulus) x ^= mul_engine(y, lm, q);
}
}  // namespace
void scalar_ifft(uint16_t *s, uint64_t size, uint64_t trunc, uint64_t sd, bool q) {
  const uint16_t *sk = tables().skew;
  uint64_t d = 1;
  for (uint64_t d4 = 4; d4 <= size; d = d4, d4 <<= 2)
    for (uint64_t r = 0; r < trunc; r += d4) {
      const uint64_t b = r + d + sd - 1;
      const uint16_t m01 = sk[b], m02 = sk[b + d], m23 = sk[b + 2 * d];
      for (uint64_t i = r; i < r + d; i++) {
        ifft_bf_s(s[i], s[i + d], m01, q);
        ifft_bf_s(s[i + 2 * d], s[i + 3 * d], m23, q);
        ifft_bf_s(s[i], s[i + 2 * d], m02, q);
        ifft_bf_s(s[i + d], s[i + 3 * d], m02, q);
      }
    }
  if (d < size) {
    const uint16_t lm = sk[d + sd - 1];
    for (uint64_t i = 0; i < d; i++) ifft_bf_s(s[i], s[d + i], lm, q);
  }
}
void scalar_fft(uint16_t *s, uint64_t size, uint64_t trunc, uint64_t sd, bool q) {
  const uint16_t *sk = tables().skew;
  uint64_t d4 = size;
  for (uint64_t d = size >> 2; d != 0; d4 = d, d >>= 2)
    for (uint64_t r = 0; r < trunc; r += d4) {
      const uint64_t b = r + d + sd - 1;
      const uint16_t m01 = sk[b], m02 = sk[b + d], m23 = sk[b + 2 * d];
      for (uint64_t i = r; i < r + d; i++) {
        fft_bf_s(s[i], s[i + 2 * d], m02, q);
        fft_bf_s(s[i + d], s[i + 3 * d], m02, q);
        fft_bf_s(s[i], s[i + d], m01, q);
        fft_bf_s(s[i + 2 * d], s[i + 3 * d], m23, q);
      }
    }
  if (d4 == 2)
    for (uint64_t r = 0; r < trunc; r += 2) fft_bf_s(s[r], s[r + 1], sk[r + sd], q);
}

namespace {
// g_logs_fwht: erasure_logs* always take the two transforms (rs_debug_erasure_logs_check)
std::atomic<bool> g_logs_fwht{false};

// eval_poly on an erasure indicator is the dyadic convolution er[i] = sum over erased j of
// log[i ^ j] (mod 65535; log[0] = 65535 adds nothing): the 65536-point transform of the
// indicator times log_walsh, transformed back, 65536 = 1 (mod 65535). A plan reads er at
// positions below W = ceilPow2(end) only, so a small erased set is summed point by point
// there (c4: 512 points x 64 terms, ~10 us, against ~1.1 ms for the two transforms on a
// first call's critical path); entries past W stay 0. Values agree with the transforms' mod
// 65535 (0 and 65535 are the same log to every consumer: exp[65535] = exp[0], add_mod).
void erasure_logs_of(uint16_t *er, uint64_t trunc, uint64_t W) {
  if (!g_logs_fwht.load(std::memory_order_relaxed)) {
    std::vector<uint32_t> ind;
    for (uint64_t j = 0; j < trunc; j++)
      if (er[j]) ind.push_back(static_cast<uint32_t>(j));
    if (W * ind.size() <= (1u << 21)) {
      const uint16_t *lg = tables().log;
      for (uint64_t i = 0; i < W; i++) {
        uint64_t sum = 0;
        for (uint32_t j : ind) sum += lg[i ^ j];
        er[i] = static_cast<uint16_t>(sum % kModulus);
      }
      return;
    }
  }
  eval_poly(er, trunc);
}
}  // namespace

void set_erasure_logs_fwht(bool on) { g_logs_fwht.store(on); }

void erasure_logs(const uint8_t *received, uint64_t k, uint64_t m, uint16_t *er) {
  const uint64_t C = ceil_pow2(m), end = C + k;
  std::memset(er, 0, kOrder * sizeof(uint16_t));
  for (uint64_t i = 0; i < m; i++)
    if (!received[i]) er[i] = 1;
  for (uint64_t i = m; i < C; i++) er[i] = 1;
  for (uint64_t i = C; i < end; i++)
    if (!received[i]) er[i] = 1;
  erasure_logs_of(er, end, ceil_pow2(end));
}

void scalar_reconstruct(uint16_t *sym, const uint8_t *received, const uint16_t *er, uint64_t k, uint64_t m,
                        bool q) {
  const uint64_t C = ceil_pow2(m), end = C + k, W = ceil_pow2(C + k);
  for (uint64_t i = 0; i < W; i++) {
    const bool live = (i < m || (i >= C && i < end)) && received[i];
    sym[i] = live ? mul_engine(sym[i], er[i], q) : 0;
  }
  scalar_ifft(sym, W, end, 0, q);
  for (uint64_t i = 1; i < W; i++) {
    const uint64_t w = i & (~i + 1);
    for (uint64_t j = 0; j < w; j++) sym[i - w + j] ^= sym[i + j];
  }
  scalar_fft(sym, W, end, 0, q);
  for (uint64_t i = C; i < end; i++)
    if (!received[i]) sym[i] = mul_engine(sym[i], static_cast<uint16_t>(kModulus - er[i]), q);
}

std::vector<uint64_t> encode_chunk_truncs(uint64_t k, uint64_t m, bool quirk_d2) {
  const uint64_t C = ceil_pow2(m);
  std::vector<uint64_t> truncs;  // chunk j at position j*C
  truncs.push_back(std::min(k, C));
  if (k > C) {
    uint64_t cs = C;
    while (quirk_d2 ? (cs + C < k) : (cs + C <= k)) {  // root.zig:151 (D2: `<`)
      truncs.push_back(C);
      cs += C;
    }
    if (k % C) truncs.push_back(k % C);  // root.zig:159-166
  }
  return truncs;
}

void scalar_encode(const uint16_t *in, uint64_t k, uint64_t m, bool quirk_d1, bool quirk_d2, uint16_t *out) {
  const uint64_t C = ceil_pow2(m);
  const std::vector<uint64_t> truncs = encode_chunk_truncs(k, m, quirk_d2);
  std::vector<uint16_t> acc(C, 0), tmp(C);
  for (size_t j = 0; j < truncs.size(); j++) {
    for (uint64_t i = 0; i < C; i++) tmp[i] = j * C + i < k ? in[j * C + i] : 0;  // zero fill, root.zig:161
    scalar_ifft(tmp.data(), C, truncs[j], (j + 1) * C, quirk_d1);  // root.zig:143-166
    for (uint64_t i = 0; i < C; i++) acc[i] ^= tmp[i];
  }
  scalar_fft(acc.data(), C, m, 0, quirk_d1);  // root.zig:169
  for (uint64_t i = 0; i < m; i++) out[i] = acc[i];
}

void scalar_encode_low(const uint16_t *in, uint64_t k, uint64_t m, bool quirk_d1, uint16_t *out) {
  const uint64_t C = ceil_pow2(k);
  std::vector<uint16_t> coef(C, 0), tmp(C);
  for (uint64_t i = 0; i < k; i++) coef[i] = in[i];
  scalar_ifft(coef.data(), C, k, 0, quirk_d1);  // originals at positions [0, k)
  for (uint64_t cs = 0; cs < m; cs += C) {       // recovery chunk at positions [C + cs, ...)
    tmp = coef;
    const uint64_t t = std::min(C, m - cs);
    scalar_fft(tmp.data(), C, t, cs + C, quirk_d1);
    for (uint64_t i = 0; i < t; i++) out[cs + i] = tmp[i];
  }
}

void erasure_logs_low(const uint8_t *received, uint64_t k, uint64_t m, uint16_t *er) {
  const uint64_t C = ceil_pow2(k), end = C + m, W = ceil_pow2(end);
  std::memset(er, 0, kOrder * sizeof(uint16_t));
  for (uint64_t i = 0; i < k; i++)
    if (!received[i]) er[i] = 1;  // missing originals; [k, C) are known zeros
  for (uint64_t i = C; i < end; i++)
    if (!received[i]) er[i] = 1;  // missing recovery
  for (uint64_t i = end; i < W; i++) er[i] = 1;  // P's values past the code: unknown
  erasure_logs_of(er, W, W);
}

void scalar_reconstruct_low(uint16_t *sym, const uint8_t *received, const uint16_t *er, uint64_t k, uint64_t m) {
  const uint64_t C = ceil_pow2(k), end = C + m, W = ceil_pow2(end);
  for (uint64_t i = 0; i < W; i++) {
    const bool live = (i < k || (i >= C && i < end)) && received[i];
    sym[i] = live ? mul16(sym[i], er[i]) : 0;
  }
  scalar_ifft(sym, W, end, 0, false);
  for (uint64_t i = 1; i < W; i++) {
    const uint64_t w = i & (~i + 1);
    for (uint64_t j = 0; j < w; j++) sym[i - w + j] ^= sym[i + j];
  }
  scalar_fft(sym, W, k, 0, false);
  for (uint64_t i = 0; i < k; i++)
    if (!received[i]) sym[i] = mul16(sym[i], static_cast<uint16_t>(kModulus - er[i]));
}

RsTab make_twiddle(uint32_t skew_index, bool quirk_d1) {
  if (skew_index >= kModulus) {  // beyond the table: only reachable for groups the device skips
    RsTab z{};
    z.flags = kTabXorOnly;
    z.log_m = kModulus;
    return z;
  }
  const uint16_t lm = tables().skew[skew_index];
  if (lm == kModulus) {
    RsTab z{};
    z.flags = kTabXorOnly;
    z.log_m = kModulus;
    return z;
  }
  return make_tab(lm, quirk_d1);
}

void fwht(uint16_t *d, uint64_t m) {
  uint64_t dist = 1, stride = 4;
  while (stride <= kOrder) {
    for (uint64_t r = 0; r < m; r += stride) {
      for (uint64_t o = r; o < r + dist; o++) {
        // walsh_hadamard.zig:38-62 (fwht4 of two fwht2 layers); offset/stride are u16 there
        const uint64_t x0 = static_cast<uint16_t>(o), st = static_cast<uint16_t>(dist);
        const uint64_t x1 = x0 + st, x2 = x0 + 2 * st, x3 = x0 + 3 * st;
        const uint16_t s0 = add_mod(d[x0], d[x1]), d0 = sub_mod(d[x0], d[x1]);
        const uint16_t s1 = add_mod(d[x2], d[x3]), d1 = sub_mod(d[x2], d[x3]);
        d[x0] = add_mod(s0, s1);
        d[x1] = add_mod(d0, d1);
        d[x2] = sub_mod(s0, s1);
        d[x3] = sub_mod(d0, d1);
      }
    }
    dist = stride;
    stride *= 4;
  }
}

void eval_poly(uint16_t *e, uint64_t truncated_size) {
  const Tables &t = tables();
  fwht(e, truncated_size);
  for (uint32_t i = 0; i < kOrder; i++) {
    const uint32_t p = static_cast<uint32_t>(e[i]) * t.log_walsh[i];
    e[i] = add_mod(p & 0xFFFF, p >> 16);
  }
  fwht(e, kOrder);
}

size_t ifft_tab_count(uint64_t size) {
  size_t n = 0;
  uint64_t d = 1, d4 = 4;
  for (; d4 <= size; d = d4, d4 <<= 2) n += 3 * (size / d4);
  if (d < size) n += 1;
  return n;
}

size_t fft_tab_count(uint64_t size) {
  size_t n = 0;
  uint64_t d = size >> 2, d4 = size;
  for (; d != 0; d4 = d, d >>= 2) n += 3 * (size / d4);
  if (d4 == 2) n += size / 2;
  return n;
}

void push_ifft_tabs(std::vector<RsTab> &out, uint64_t size, uint64_t sd, bool q) {
  uint64_t d = 1, d4 = 4;
  for (; d4 <= size; d = d4, d4 <<= 2) {
    for (uint64_t r = 0; r < size; r += d4) {
      const uint64_t base = r + d + sd - 1;  // Generic.zig:88-92
      out.push_back(make_twiddle(static_cast<uint32_t>(base), q));          // m01
      out.push_back(make_twiddle(static_cast<uint32_t>(base + d), q));      // m02
      out.push_back(make_twiddle(static_cast<uint32_t>(base + 2 * d), q));  // m23
    }
  }
  if (d < size) out.push_back(make_twiddle(static_cast<uint32_t>(d + sd - 1), q));  // Generic.zig:131-132
}

void push_fft_tabs(std::vector<RsTab> &out, uint64_t size, uint64_t sd, bool q) {
  uint64_t d = size >> 2, d4 = size;
  for (; d != 0; d4 = d, d >>= 2) {
    for (uint64_t r = 0; r < size; r += d4) {
      const uint64_t base = r + d + sd - 1;  // Generic.zig:23-27
      out.push_back(make_twiddle(static_cast<uint32_t>(base), q));
      out.push_back(make_twiddle(static_cast<uint32_t>(base + d), q));
      out.push_back(make_twiddle(static_cast<uint32_t>(base + 2 * d), q));
    }
  }
  if (d4 == 2)  // Generic.zig:64-77
    for (uint64_t r = 0; r < size; r += 2) out.push_back(make_twiddle(static_cast<uint32_t>(r + sd), q));
}

}  // namespace rs
