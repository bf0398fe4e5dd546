// rs_fftnet.cpp — generator and launcher of the bit-sliced additive-FFT encode
// kernels (rs_fftnet.hpp).
#include "rs_fftnet.hpp"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <sstream>

#include "reedsol.h"
#include "rs_gf.hpp"
#include "rs_internal.hpp"

namespace rs {
namespace fftnet {
namespace {

// ------------------------------------------------------------------ field side
// T: Cantor coordinates (lo = beta_0..7, hi = beta_8..15) -> (u, v) with
// x = u + beta_8 * v, u, v in GF(2^8) = span(beta_0..beta_7) (a Cantor basis spans
// subfields, gf.zig:8-13). beta_{8+i} = p_i + beta_8 * beta_i, so v = hi and
// u = lo ^ sum_i hi_i p_i; T is an involution.
struct Basis {
  bool ok = false;
  uint8_t p[8] = {};
};

const Basis &basis() {
  static const Basis b = [] {
    Basis r;
    const Tables &t = tables();
    r.ok = true;
    for (int i = 0; i < 8; i++) {
      const uint16_t prod = mul16(static_cast<uint16_t>(1u << 8), t.log[1u << i]);  // beta_8 * beta_i
      const uint16_t pi = static_cast<uint16_t>((1u << (8 + i)) ^ prod);
      if (pi >> 8) r.ok = false;
      r.p[i] = static_cast<uint8_t>(pi);
    }
    return r;
  }();
  return b;
}

uint16_t to_uv(uint16_t x) {
  const Basis &b = basis();
  uint8_t lo = 0;
  for (int i = 0; i < 8; i++)
    if (x >> (8 + i) & 1) lo ^= b.p[i];
  return static_cast<uint16_t>(x ^ lo);
}

// A twiddle's multiply in (u, v) coordinates: u' = A u + B v, v' = Cm u + D v
// (row masks: bit j of A[i] = u-input j feeds u-output i). Subfield twiddles have
// B = Cm = 0 and A = D.
struct Tw {
  bool zero = true;  // log 65535: XOR-only butterfly (Generic.zig:38,47,53,103,...)
  bool sub = false;
  uint8_t A[8] = {}, B[8] = {}, Cm[8] = {}, D[8] = {};
};

Tw twiddle(uint16_t log_m, bool d1) {
  Tw t;
  if (log_m == kModulus) return t;
  t.zero = false;
  for (int j = 0; j < 8; j++) {
    const uint16_t cu = to_uv(mul_engine(to_uv(static_cast<uint16_t>(1u << j)), log_m, d1));
    const uint16_t cv = to_uv(mul_engine(to_uv(static_cast<uint16_t>(1u << (8 + j))), log_m, d1));
    for (int i = 0; i < 8; i++) {
      t.A[i] |= static_cast<uint8_t>((cu >> i & 1) << j);
      t.Cm[i] |= static_cast<uint8_t>((cu >> (8 + i) & 1) << j);
      t.B[i] |= static_cast<uint8_t>((cv >> i & 1) << j);
      t.D[i] |= static_cast<uint8_t>((cv >> (8 + i) & 1) << j);
    }
  }
  t.sub = true;
  for (int i = 0; i < 8; i++)
    if (t.B[i] || t.Cm[i] || t.A[i] != t.D[i]) t.sub = false;
  return t;
}

// --------------------------------------------------------------- the schedule
struct Bf {
  uint32_t x, y;
  uint16_t log_m;
};
struct Layer {
  int bit;
  bool inv;  // IFFT butterfly (y ^= x; x ^= M y) or FFT (x ^= M y; y ^= x)
  std::vector<Bf> bf;
};

uint16_t sk(uint64_t idx) { return idx < kModulus ? tables().skew[idx] : static_cast<uint16_t>(kModulus); }

uint16_t gmul_elem(uint16_t x, uint16_t y) { return x && y ? mul16(x, tables().log[y]) : 0; }

int log2i(uint64_t v) {
  int b = 0;
  while ((1ull << b) < v) b++;
  return b;
}

// Generic.zig:80-147, group for group (groups r >= trunc skipped as there)
std::vector<Layer> ifft_layers(uint64_t size, uint64_t trunc, uint64_t sd) {
  std::vector<Layer> out;
  uint64_t d = 1;
  for (uint64_t d4 = 4; d4 <= size; d = d4, d4 <<= 2) {
    Layer l1{log2i(d), true, {}}, l2{log2i(d) + 1, true, {}};
    for (uint64_t r = 0; r < trunc; r += d4) {
      const uint64_t b = r + d + sd - 1;
      const uint16_t m01 = sk(b), m02 = sk(b + d), m23 = sk(b + 2 * d);
      for (uint64_t i = r; i < r + d; i++) {
        l1.bf.push_back({uint32_t(i), uint32_t(i + d), m01});
        l1.bf.push_back({uint32_t(i + 2 * d), uint32_t(i + 3 * d), m23});
        l2.bf.push_back({uint32_t(i), uint32_t(i + 2 * d), m02});
        l2.bf.push_back({uint32_t(i + d), uint32_t(i + 3 * d), m02});
      }
    }
    out.push_back(std::move(l1));
    out.push_back(std::move(l2));
  }
  if (d < size) {  // final odd layer, Generic.zig:131-146
    Layer l{log2i(d), true, {}};
    const uint16_t lm = sk(d + sd - 1);
    for (uint64_t i = 0; i < d; i++) l.bf.push_back({uint32_t(i), uint32_t(d + i), lm});
    out.push_back(std::move(l));
  }
  return out;
}

// Generic.zig:15-78
std::vector<Layer> fft_layers(uint64_t size, uint64_t trunc, uint64_t sd) {
  std::vector<Layer> out;
  uint64_t d4 = size;
  for (uint64_t d = size >> 2; d != 0; d4 = d, d >>= 2) {
    Layer l1{log2i(d) + 1, false, {}}, l2{log2i(d), false, {}};
    for (uint64_t r = 0; r < trunc; r += d4) {
      const uint64_t b = r + d + sd - 1;
      const uint16_t m01 = sk(b), m02 = sk(b + d), m23 = sk(b + 2 * d);
      for (uint64_t i = r; i < r + d; i++) {
        l1.bf.push_back({uint32_t(i), uint32_t(i + 2 * d), m02});
        l1.bf.push_back({uint32_t(i + d), uint32_t(i + 3 * d), m02});
        l2.bf.push_back({uint32_t(i), uint32_t(i + d), m01});
        l2.bf.push_back({uint32_t(i + 2 * d), uint32_t(i + 3 * d), m23});
      }
    }
    out.push_back(std::move(l1));
    out.push_back(std::move(l2));
  }
  if (d4 == 2) {  // Generic.zig:64-77
    Layer l{0, false, {}};
    for (uint64_t r = 0; r < trunc; r += 2) l.bf.push_back({uint32_t(r), uint32_t(r + 1), sk(r + sd)});
    out.push_back(std::move(l));
  }
  return out;
}

// ------------------------------------------------------------------- the plan
// Positions of a chunk: n = log2(C) bits. Layout A: wave = p >> 3, reg = p & 7
// (bits 0..2 in registers). Layout B: wave = p & (NW - 1), reg = p >> WB.
struct Plan {
  uint32_t k = 0, m = 0, C = 0, n = 0, WB = 0, NW = 0;
  bool d1 = false;
  std::vector<uint64_t> truncs;
  std::vector<std::vector<Layer>> ifft;  // per chunk
  std::vector<Layer> fft;
  std::vector<std::vector<uint8_t>> valid;  // [chunk][p]: data shard present (not padding, not skipped)
  std::vector<uint8_t> out_mode;            // [p < C]
  std::map<uint16_t, Tw> tw;

  uint32_t waveA(uint32_t p) const { return p >> 3; }
  uint32_t regA(uint32_t p) const { return p & 7; }
  uint32_t waveB(uint32_t p) const { return p & (NW - 1); }
  uint32_t regB(uint32_t p) const { return p >> WB; }
  uint32_t posA(uint32_t w, uint32_t r) const { return (w << 3) | r; }
  uint32_t posB(uint32_t w, uint32_t t) const { return (t << WB) | w; }
  bool inA(int bit) const { return bit < 3; }
  const Tw &get_tw(uint16_t l) {
    auto it = tw.find(l);
    if (it == tw.end()) it = tw.emplace(l, twiddle(l, d1)).first;
    return it->second;
  }
};

Plan make_plan(const Spec &s) {
  Plan p;
  p.k = s.k;
  p.m = s.m;
  p.C = static_cast<uint32_t>(ceil_pow2(s.m));
  p.n = static_cast<uint32_t>(log2i(p.C));
  p.WB = p.n - 3;
  p.NW = 1u << p.WB;
  p.d1 = (s.flags & RS_FLAG_QUIRK_D1) != 0;
  // inverse: parity = FFT_0(IFFT_C(data)) for k == m == C (no truncation, D2 cannot
  // drop the only chunk), so data = FFT_C(IFFT_0(parity)): each butterfly layer of one
  // skew undoes the other's (Generic.zig:15-147), under either multiply
  p.truncs = s.inverse ? std::vector<uint64_t>{p.C} : encode_chunk_truncs(s.k, s.m, (s.flags & RS_FLAG_QUIRK_D2) != 0);
  for (size_t j = 0; j < p.truncs.size(); j++) {
    p.ifft.push_back(ifft_layers(p.C, p.truncs[j], s.inverse ? 0 : (j + 1) * p.C));  // root.zig:143-166
    std::vector<uint8_t> v(p.C, 0);
    for (uint32_t q = 0; q < p.C; q++) {
      const uint64_t g = j * p.C + q;
      v[q] = g < s.k && !(g < s.skip.size() && s.skip[g]) && !(g < s.present.size() && !s.present[g]);
    }
    p.valid.push_back(std::move(v));
  }
  p.fft = fft_layers(p.C, s.inverse ? s.k : s.m, s.inverse ? p.C : 0);  // root.zig:169
  p.out_mode.assign(p.C, kOutNone);
  for (uint32_t q = 0; q < s.m; q++) p.out_mode[q] = s.out_mode.empty() ? kOutStore : s.out_mode[q];
  if (!s.present.empty()) {  // static decode: Enc(d') is needed on the rows R only
    uint32_t e = 0, nr = 0;
    for (uint32_t g = 0; g < s.k; g++) e += s.present[g] ? 0 : 1;
    for (uint32_t q = 0; q < s.m; q++) {
      const bool in_r = s.present[s.k + q] && nr < e;
      nr += in_r ? 1 : 0;
      p.out_mode[q] = in_r ? kOutStore : kOutNone;
    }
  }
  return p;
}

// ------------------------------------------------------------------ code gen
const char *kPrelude = R"HIP(
typedef unsigned int u32;
typedef unsigned long long u64;
typedef u32 v4 __attribute__((ext_vector_type(4)));
#define X3(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)
#define MUX(a, b, m) __builtin_amdgcn_bitop3_b32((a), (b), (m), 0xE4)
// the nibble / bit-pair / bit masks: in VGPRs when RS_VMASK (a VALU instruction that
// reads an SGPR issues at ~2/3 rate when two waves share the SIMD: 3.67 vs 2.67 cycles per
// v_bitop3, profiles/r04/valu_probe2.log), else literals the compiler keeps in SGPRs
struct Km {
  u32 f, t, s;
};
#define XM(d, n) __builtin_amdgcn_bitop3_b32((d), (n), KM.f, 0x78)
#define SWN(a) MUX((a) >> 4, (a) << 4, KM.f)
#define TRS(j, d, m)                 \
  {                                  \
    const u32 a = x[j], b = x[j + d]; \
    x[j] = MUX(a, b << d, m);        \
    x[j + d] = MUX(a >> d, b, m);    \
  }
__device__ __forceinline__ void tr8(u32 *x, const Km KM) {
  TRS(0, 4, KM.f) TRS(1, 4, KM.f) TRS(2, 4, KM.f) TRS(3, 4, KM.f)
  TRS(0, 2, KM.t) TRS(1, 2, KM.t) TRS(4, 2, KM.t) TRS(5, 2, KM.t)
  TRS(0, 1, KM.s) TRS(2, 1, KM.s) TRS(4, 1, KM.s) TRS(6, 1, KM.s)
}
// raw buffer accesses: voffset = the lane's offset in the unit, soffset = the
// (wave-uniform) shard offset; a resource with 0 records reads zeros
#define LDB(r, vo, so) __builtin_amdgcn_raw_buffer_load_b128((r), (vo), (so), RS_AUX_LD)
// A 128-bit store's data registers must not be rewritten by the next instruction: LLVM
// inserts that wait state for buffer stores only when soffset is not a register, and a
// build whose next VALU overwrote the first data dword stored that value in lanes 12-15
// of every row (profiles/r03/spill_root_cause.md). The s_nop reads the data, so the
// registers stay live until it has issued: at least one wait state, whatever the schedule.
#define STB(v, r, vo, so)                                                      \
  {                                                                            \
    const v4 sv_ = (v);                                                        \
    __builtin_amdgcn_raw_buffer_store_b128(sv_, (r), (vo), (so), RS_AUX_ST);   \
    asm volatile("s_nop 0" ::"v"(sv_) : "memory");                             \
  }
// 2 KiB slice of a shard: lanes 0-31 read the lo halves, 32-63 the hi halves of
// 16 chunks per KiB; one v_permlane32_swap per dword pairs them; then an 8x8 bit
// transpose per byte lane: P[j] = (lo plane j | hi plane j) per byte (nibbles)
__device__ __forceinline__ void planes2(v4 a, v4 b, u32 *P, const Km KM) {
#pragma unroll
  for (int v = 0; v < 4; v++) {
    const auto s = __builtin_amdgcn_permlane32_swap(a[v], b[v], false, false);
    P[v] = s[0];
    P[4 + v] = s[1];
  }
  tr8(P, KM);
}
__device__ __forceinline__ void unplanes2(u32 *P, v4 &a, v4 &b, const Km KM) {
  tr8(P, KM);
#pragma unroll
  for (int v = 0; v < 4; v++) {
    const auto s = __builtin_amdgcn_permlane32_swap(P[v], P[4 + v], false, false);
    a[v] = s[0];
    b[v] = s[1];
  }
}
// LDS exchange: slot s = 2 KiB (8 planes x 64 lanes), xch[lq + (s * 8 + i) * 64] holds
// plane i (dword accesses: no 4-register tuples to assemble); lq = lane, laundered at
// every exchange so the compiler keeps one base register instead of hoisting an
// address per slot out of the unit loop
#define LQ()      \
  u32 lq = lane; \
  asm volatile("" : "+v"(lq));
#define BAR()                                                      \
  {                                                                \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local"); \
    __builtin_amdgcn_s_barrier();                                  \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local"); \
  }
// RS_AMD_FFT_DEBUG bit 6 (measurement builds): lane 0 of every wave of workgroup 0 stamps
// s_memtime around each barrier of its third unit into stamps[w * 64 + i]
#define STAMP(i)                                                         \
  if (RS_STAMPS && stamp_on && lane == 0u) {                             \
    asm volatile("" ::: "memory");                                       \
    stamps[w * 64u + (i)] = __builtin_amdgcn_s_memtime();                \
    asm volatile("" ::: "memory");                                       \
  }
// Spec::decode: multiplication by a uniform runtime scalar from its 128 nibble masks
// (scalar_masks), read through the constant address space (scalar loads):
// out_i = XOR_j (x_j & M[16 i + j]) ^ (SWN(x_j) & M[16 i + 8 + j])
typedef const __attribute__((address_space(4))) u32 *cptr;
// RS_RMUL_G output planes per step: their 16 G masks are read together (one scalar-load
// wait per step instead of per plane) and their chains interleave
#ifndef RS_RMUL_G
#define RS_RMUL_G 1
#endif
__device__ __forceinline__ void rmul(u32 *x, cptr M, const Km KM) {
#ifdef RS_DBG_NORMUL
  return;
#endif
  u32 s[8], o[8];
#pragma unroll
  for (int j = 0; j < 8; j++) s[j] = SWN(x[j]);
#pragma unroll
  for (int i0 = 0; i0 < 8; i0 += RS_RMUL_G) {
    u32 m[16 * RS_RMUL_G];
#pragma unroll
    for (int t = 0; t < 16 * RS_RMUL_G; t++) m[t] = M[16 * i0 + t];
#pragma unroll
    for (int g = 0; g < RS_RMUL_G; g++) {
      u32 a = x[0] & m[16 * g];
#pragma unroll
      for (int j = 1; j < 8; j++) a = __builtin_amdgcn_bitop3_b32(a, x[j], m[16 * g + j], 0x78);
#pragma unroll
      for (int j = 0; j < 8; j++) a = __builtin_amdgcn_bitop3_b32(a, s[j], m[16 * g + 8 + j], 0x78);
      o[i0 + g] = a;
    }
  }
#pragma unroll
  for (int i = 0; i < 8; i++) x[i] = o[i];
}
)HIP";

int env_int(const char *name, int def) {
  const char *e = std::getenv(name);
  return e && *e ? std::atoi(e) : def;
}


// butterflies between sched_barriers: 0 / 2 / 4 measured the same as 1 (RS(200,55) encode
// 3.72 / 3.70 / 3.72 vs 3.69 ms, fused decode 6.86 / 6.89 / 6.89 vs 6.90 ms,
// profiles/r03/negative/fft_sched_spacing.jsonl); 1 bounds the compile time
int sched_of() { return 1; }

int prefetch_of(const Spec &s) {
  return std::max(0, std::min(8, s.prefetch >= 0 ? s.prefetch : env_int("RS_AMD_FFT_PREFETCH", 4)));
}

// RS_AMD_FFT_DEBUG (measurement builds only, part of the cache key): bit 0 loads read
// through the zero-record resource (no HBM reads), bit 1 stores dropped the same way, bit 2
// decode kernels stop after Enc(d') (no decode tail), bit 3 decode: no runtime multiplies,
// bit 4 decode: the round-3 load order (rec rows loaded at the tail, no prefetch)
int debug_of() { return env_int("RS_AMD_FFT_DEBUG", 0); }

// the stamp buffer of measurement builds (8 waves x 64 u64 per device)
std::mutex g_stamp_mu;
std::map<int, unsigned long long *> g_stamp_bufs;
unsigned long long *stamp_buffer(int dev) {
  std::lock_guard<std::mutex> lk(g_stamp_mu);
  unsigned long long *&p = g_stamp_bufs[dev];
  if (!p && hipMalloc(reinterpret_cast<void **>(&p), 8 * 64 * 8) == hipSuccess) (void)hipMemset(p, 0, 8 * 64 * 8);
  return p;
}

// Spec::present: where a wave's rows of R are loaded (RS_AMD_PDEC_RLOAD): 0 at the start of its
// syndrome branch (round 4), 1 at the start of its final-FFT A layers (in flight during them),
// 2 before the final FFT's B layers (round 4's dbg bit 5), 3 half at 1, half at 0
int rload_of() {
  const int v = env_int("RS_AMD_PDEC_RLOAD", 0);
  return v >= 0 && v <= 3 ? v : 0;
}

// unit walk (RS_AMD_FFT_WALK): 1 = blocked (workgroup b takes units [b per, (b + 1) per): a
// stripe's 2 KiB column slices in order, each shard row streamed sequentially by one CU),
// 0 = interleaved (units b, b + grid, ...: every CU on the same two stripes at once)
int walk_of() { return env_int("RS_AMD_FFT_WALK", 0) ? 1 : 0; }

// the transpose / basis masks in VGPRs (RS_AMD_FFT_VMASK, default on)
int vmask_of() { return env_int("RS_AMD_FFT_VMASK", 1) ? 1 : 0; }

// runtime-multiply output planes per scalar-load step (RS_AMD_FFT_RMULG: 1, 2, 4, 8). 4: per-stripe
// RS(200,55) max_e 55 7.35 -> 6.66 ms, RS(16,16) 2.79 -> 2.71 ms (profiles/r04/patterns/rmul_ab.log).
// Measured and removed: the masks through vector loads (7.35 -> 8.9 ms), s_setprio turns
// between the SIMD-pair halves (c4 neutral to 8 % slower, profiles/r04/prio1.log)
int rmul_group() {
  const int g = env_int("RS_AMD_FFT_RMULG", 4);
  return g == 2 || g == 4 || g == 8 ? g : 1;
}

struct Gen {
  std::ostringstream o;
  int tmp = 0;
  Stats *st = nullptr;
  uint64_t *ops = nullptr;  // counter the current section adds to

  std::string fresh(const char *p = "zt") { return p + std::to_string(tmp++); }
  void op(uint64_t n = 1) {
    if (ops) *ops += n;
  }

  // dst[i] (^)= XOR over j in rows[i] of ins[j]; pairs shared by >= 2 rows are
  // built once (Paar's greedy), each row is then an XOR3 chain.
  void rows(const std::vector<std::string> &ins, const std::vector<uint32_t> &rowmask,
            const std::vector<std::string> &dst, bool acc) {
    std::vector<std::string> names = ins;
    std::vector<std::vector<int>> r(rowmask.size());
    for (size_t i = 0; i < rowmask.size(); i++)
      for (size_t j = 0; j < ins.size(); j++)
        if (rowmask[i] >> j & 1) r[i].push_back(static_cast<int>(j));
    for (;;) {
      std::map<std::pair<int, int>, int> cnt;
      for (auto &row : r)
        for (size_t a = 0; a < row.size(); a++)
          for (size_t b = a + 1; b < row.size(); b++) cnt[{std::min(row[a], row[b]), std::max(row[a], row[b])}]++;
      std::pair<int, int> best{-1, -1};
      int bc = 1;
      for (auto &kv : cnt)
        if (kv.second > bc) {
          bc = kv.second;
          best = kv.first;
        }
      if (best.first < 0) break;
      const std::string nm = fresh();
      o << "  const u32 " << nm << " = " << names[best.first] << " ^ " << names[best.second] << ";\n";
      op();
      const int id = static_cast<int>(names.size());
      names.push_back(nm);
      for (auto &row : r) {
        auto ia = std::find(row.begin(), row.end(), best.first), ib = std::find(row.begin(), row.end(), best.second);
        if (ia != row.end() && ib != row.end()) {
          row.erase(std::remove_if(row.begin(), row.end(), [&](int v) { return v == best.first || v == best.second; }),
                    row.end());
          row.push_back(id);
        }
      }
    }
    for (size_t i = 0; i < r.size(); i++) {
      std::vector<std::string> t;
      for (int id : r[i]) t.push_back(names[id]);
      const std::string &d = dst[i];
      size_t at = 0;
      if (!acc) {
        if (t.empty()) {
          o << "  " << d << " = 0u;\n";
          continue;
        }
        if (t.size() == 1) {
          o << "  " << d << " = " << t[0] << ";\n";
          continue;
        }
        if (t.size() == 2 || t.size() == 4) {
          o << "  " << d << " = " << t[0] << " ^ " << t[1] << ";\n";
          at = 2;
        } else {
          o << "  " << d << " = X3(" << t[0] << ", " << t[1] << ", " << t[2] << ");\n";
          at = 3;
        }
        op();
      }
      for (; at + 1 < t.size(); at += 2) {
        o << "  " << d << " = X3(" << d << ", " << t[at] << ", " << t[at + 1] << ");\n";
        op();
      }
      if (at < t.size()) {
        o << "  " << d << " ^= " << t[at] << ";\n";
        op();
      }
    }
  }

  static std::vector<std::string> regs(const std::string &pfx) {
    std::vector<std::string> v;
    for (int i = 0; i < 8; i++) v.push_back(pfx + "_" + std::to_string(i));
    return v;
  }

  // dst (^)= M(src) for a twiddle
  void mul(const std::vector<std::string> &dst, bool acc, const std::vector<std::string> &src, const Tw &t) {
    if (t.sub) {
      if (st) st->subfield++;
      std::vector<uint32_t> rm(8);
      for (int i = 0; i < 8; i++) rm[i] = t.A[i];
      rows(src, rm, dst, acc);
      return;
    }
    if (st) st->general++;
    // nibble-swapped copies s_j = (v_j | u_j): the low nibble of A y + B s is
    // A u + B v, the high nibble of D y + Cm s is Cm u + D v
    std::vector<std::string> ins = src;
    for (int j = 0; j < 8; j++) {
      const std::string s = fresh("zs");
      o << "  const u32 " << s << " = SWN(" << src[j] << ");\n";
      op(3);
      ins.push_back(s);
    }
    std::vector<uint32_t> rm(16);
    std::vector<std::string> tl(16);
    for (int i = 0; i < 8; i++) {
      rm[i] = t.A[i] | (uint32_t(t.B[i]) << 8);
      rm[8 + i] = t.D[i] | (uint32_t(t.Cm[i]) << 8);
      tl[i] = fresh("zl");
      tl[8 + i] = fresh("zh");
    }
    o << "  u32 ";
    for (int i = 0; i < 16; i++) o << tl[i] << (i < 15 ? ", " : ";\n");
    rows(ins, rm, tl, false);
    for (int i = 0; i < 8; i++) {
      if (acc)
        o << "  " << dst[i] << " ^= MUX(" << tl[i] << ", " << tl[8 + i] << ", KM.f);\n";
      else
        o << "  " << dst[i] << " = MUX(" << tl[i] << ", " << tl[8 + i] << ", KM.f);\n";
      op(acc ? 2 : 1);
    }
  }

  // materialise values here (no sinking of their computation past this point)
  void pin(const std::vector<std::string> &v) {
    o << "  asm volatile(\"\" :";
    for (size_t i = 0; i < v.size(); i++) o << (i ? ", " : " ") << "\"+v\"(" << v[i] << ")";
    o << ");\n";
  }

  void copy(const std::vector<std::string> &dst, const std::vector<std::string> &src) {
    for (int i = 0; i < 8; i++) o << "  " << dst[i] << " = " << src[i] << ";\n";
  }
  void xor_into(const std::vector<std::string> &dst, const std::vector<std::string> &src) {
    for (int i = 0; i < 8; i++) o << "  " << dst[i] << " ^= " << src[i] << ";\n";
    op(8);
  }

  int sched = 0;  // sched_barrier every `sched` butterflies (bounds the scheduler's interleaving)
  int nbf = 0;

  // one butterfly on named 8-dword positions with zero tracking
  void butterfly(const std::string &xn, bool &zx, const std::string &yn, bool &zy, bool inv, const Tw &t) {
    const auto X = regs(xn), Y = regs(yn);
    if (zx && zy) return;
    if (sched && ++nbf % sched == 0) o << "  __builtin_amdgcn_sched_barrier(0);\n";
    if (t.zero && st) st->xor_only++;
    if (inv) {  // ifftPartial, Generic.zig:171-192: y ^= x; x ^= M y
      if (!zx) {
        if (zy)
          copy(Y, X);
        else
          xor_into(Y, X);
        zy = false;
      }
      if (!t.zero && !zy) {
        mul(X, !zx, Y, t);
        zx = false;
      }
    } else {  // fftPartial, Generic.zig:149-169: x ^= M y; y ^= x
      if (!t.zero && !zy) {
        mul(X, !zx, Y, t);
        zx = false;
      }
      if (!zx) {
        if (zy)
          copy(Y, X);
        else
          xor_into(Y, X);
        zy = false;
      }
    }
  }

  // Cantor (lo|hi) <-> (u|v) on the 8 dwords of one position (an involution)
  void basis_change(const std::vector<std::string> &d) {
    const Basis &b = basis();
    std::vector<std::string> h(8), nn(8);
    for (int i = 0; i < 8; i++) {
      h[i] = fresh("zv");
      o << "  const u32 " << h[i] << " = " << d[i] << " >> 4;\n";
      op();
    }
    std::vector<uint32_t> rm(8, 0);
    for (int j = 0; j < 8; j++)
      for (int i = 0; i < 8; i++)
        if (b.p[i] >> j & 1) rm[j] |= 1u << i;
    o << "  u32 ";
    for (int j = 0; j < 8; j++) {
      nn[j] = fresh("zn");
      o << nn[j] << (j < 7 ? ", " : ";\n");
    }
    rows(h, rm, nn, false);
    for (int j = 0; j < 8; j++)
      if (rm[j]) {
        o << "  " << d[j] << " = XM(" << d[j] << ", " << nn[j] << ");\n";
        op();
      }
  }
};

std::string wname(uint32_t r) { return "w" + std::to_string(r); }
std::string bname(uint32_t t) { return "b" + std::to_string(t); }
std::string cname(uint32_t t) { return "c" + std::to_string(t); }

// wave-uniform 8-bit masks (one per wave) as a select chain on the wave index
std::string mask_expr(const std::vector<uint32_t> &per_wave) {
  bool same = true;
  for (uint32_t v : per_wave) same &= v == per_wave[0];
  if (same) return std::to_string(per_wave[0]) + "u";
  std::string e = "0u";
  for (size_t w = per_wave.size(); w-- > 0;)
    e = "(w == " + std::to_string(w) + "u ? " + std::to_string(per_wave[w]) + "u : " + e + ")";
  return e;
}

// Spec::dyn mask block of a stripe (u32 words): bit p of words [0, dyn_store_word) =
// data position p skipped (read as zero); bit q of the next 2 words = row q stored
uint32_t dyn_store_word(const Plan &P) { return static_cast<uint32_t>((P.truncs.size() * P.C + 31) / 32); }

std::string gen_source(const Spec &s, const std::string &name, Stats *stats) {
  Plan P = make_plan(s);
  Gen g;
  g.st = stats;
  g.sched = sched_of();  // sched_barrier per butterfly: bounds the scheduler's interleaving (compile time)
  Stats dummy;
  if (!g.st) g.st = &dummy;
  std::ostringstream &o = g.o;
  const uint32_t NW = P.NW, C = P.C;
  bool any_xor = s.decode;  // the decode reads the recovery rows R
  for (uint32_t q = 0; q < s.m; q++) any_xor |= P.out_mode[q] == kOutXorRec;
  // non-temporal loads and stores (cache policy bit nt = 2): RS(200,55) 256 KiB encode
  // 3.84 -> 3.70 ms (profiles/r02/fft_sweep_*.jsonl)
  const bool dyn = s.dyn;
  const int dbg = debug_of();
  // decode kernels: the recovery rows R are loaded before the final FFT's B layers (in
  // flight during them, the B -> A exchange and the A layers), the next unit's leading
  // chunk-0 positions before the last data block (the IFFT result is dead from there);
  // RS_AMD_FFT_DEBUG bit 4: the round-3 order (rows loaded at the tail, no prefetch)
  const bool old_order = s.decode && (dbg & 16);
  const bool tail = s.decode && !(dbg & 4);
  // Spec::present: the pattern compiled in (rows R, locator constants, outputs, blocks)
  const bool spat = s.decode && !s.present.empty();
  std::vector<uint8_t> inR(C, 0);         // recovery row p is one of the rows R
  std::vector<uint16_t> lp_log(C, 0);     // log of L_p (row p in R)
  std::vector<int32_t> out_row(s.k, -1);  // output row of erased data shard g
  std::vector<uint32_t> cg_log(s.k, 0);   // log of L'_g beta_K (kModulus + 1: zero)
  if (spat) {
    const Tables &T = tables();
    uint32_t e = 0, nr = 0;
    for (uint32_t g = 0; g < s.k; g++) e += s.present[g] ? 0 : 1;
    std::vector<uint8_t> received(ceil_pow2(C + s.k), 0);
    for (uint32_t p = 0; p < s.m && nr < e; p++)
      if (s.present[s.k + p]) received[p] = inR[p] = 1, nr++;
    for (uint32_t g = 0; g < s.k; g++) received[C + g] = s.present[g] ? 1 : 0;
    std::vector<uint16_t> er(kOrder);
    erasure_logs(received.data(), s.k, s.m, er.data());  // root.zig:277-289, as decode_block
    std::vector<uint16_t> beta;
    decode_betas(s.k, s.m, beta);
    for (uint32_t p = 0; p < s.m; p++)
      if (inR[p]) lp_log[p] = T.log[T.exp[er[p]]];  // root.zig:292-295
    int32_t row = 0;
    for (uint32_t g = 0; g < s.k; g++)
      if (!s.present[g]) {
        out_row[g] = row++;
        const uint16_t c = gmul_elem(beta[(C + g) / C], T.exp[kModulus - er[C + g]]);  // root.zig:321-326
        cg_log[g] = c ? T.log[c] : kModulus + 1u;
      }
  }
  o << "#define RS_AUX_LD 2\n#define RS_AUX_ST 2\n#define RS_STAMPS " << ((dbg & 64) ? 1 : 0) << "\n"
    << (s.decode && (dbg & 8) ? "#define RS_DBG_NORMUL 1\n" : "")
    << "#define RS_RMUL_G " << rmul_group() << "\n" << kPrelude;
  // 1 KiB shards (pieces 2): a unit's two 1 KiB halves are the same slice of stripes
  // 2u and 2u + 1 (resources R* and R*1; the second is the zero-record RZ past the
  // batch, so its loads read zeros and its stores are dropped)
  const bool two = s.pieces == 2;
  auto rsrc = [&](const char *base, const char *stride, const std::string &stripe, uint32_t rows) {
    return std::string("__builtin_amdgcn_make_buffer_rsrc((void *)(") + base + " + (" + stripe + ") * " + stride +
           "), (short)0, (int)(" + std::to_string(rows) + "u * sbl), 0x00020000)";
  };
  // name = rsrc(stripe0) [, name1 = rsrc(stripe0 + 1) or RZ]; `guard`: the unit exists
  auto rsrc_pair = [&](std::ostream &os_, const char *name, const char *base, const char *stride, const std::string &st0,
                       uint32_t rows, const std::string &guard) {
    const std::string nm = name;
    if (((dbg & 1) && (nm == "RD" || nm == "RR" || nm == "RDn")) || ((dbg & 2) && nm == "RO")) {  // measurement builds
      os_ << "  const __amdgpu_buffer_rsrc_t " << name << " = RZ, " << name << "1 = RZ;\n";
      return;
    }
    const std::string s0 = two ? "(" + st0 + ") * 2u" : st0;
    os_ << "  const __amdgpu_buffer_rsrc_t " << name << " = " << (guard.empty() ? "" : guard + " ? ")
        << rsrc(base, stride, s0, rows) << (guard.empty() ? "" : " : RZ") << ";\n";
    if (two)
      os_ << "  const __amdgpu_buffer_rsrc_t " << name << "1 = " << (guard.empty() ? "" : guard + " && ") << s0
          << " + 1u < n_st ? " << rsrc(base, stride, s0 + " + 1u", rows) << " : RZ;\n";
    else
      os_ << "  const __amdgpu_buffer_rsrc_t " << name << "1 = " << name << ";\n";
  };
  const char *half = two ? "loff" : "uo + 1024u";  // offset of a unit's second KiB
  o << "extern \"C\" __global__ __launch_bounds__(" << NW * 64 << ") void " << name
    << "(const unsigned char *__restrict__ data, u64 ds, const unsigned char *__restrict__ rec, u64 rs,\n"
       "    unsigned char *__restrict__ out, u64 os, u32 sb, u32 ups, u64 n_units, u64 n_st,\n"
       "    const u32 *__restrict__ dm, u32 dmw, u64 *__restrict__ stamps) {\n"
    << "  __shared__ u32 xch[" << C * 8 * 64 << "];\n"
    << "  v4 *const xch4 = (v4 *)xch;\n"
    << "  Km KM = {0x0F0F0F0Fu, 0x33333333u, 0x55555555u};\n"
    << (vmask_of() ? "  asm volatile(\"\" : \"+v\"(KM.f), \"+v\"(KM.t), \"+v\"(KM.s));\n" : "")
    << "  const u32 lane = threadIdx.x & 63u, ll = lane & 31u;\n"
       "  const u32 w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n"
       "  const u32 loff = (ll >> 1) * 64u + (lane >= 32u ? 32u : 0u) + (ll & 1u) * 16u;\n"
       // unit u = stripe * ups + uu, walked with SALU counters (no 64-bit division in the loop)
    << (s.blocked ?
       // blocked walk: workgroup b takes units [b per, (b + 1) per), a stripe's units in a row
       // (per-stripe decode blocks stay in the scalar cache)
       "  const u64 per = (n_units + gridDim.x - 1) / gridDim.x, ub = (u64)blockIdx.x * per,\n"
       "            ue = ub + per < n_units ? ub + per : n_units, step = 1;\n"
       "  u64 stripe = ub / ups;\n"
       "  u32 uu = (u32)(ub - stripe * ups);\n"
       "  const u32 gdiv = 0, gmod = 1;\n" :
       "  const u64 ub = blockIdx.x, ue = n_units, step = gridDim.x;\n"
       "  u64 stripe = blockIdx.x / ups;\n"
       "  u32 uu = blockIdx.x - (u32)stripe * ups;\n"
       "  const u32 gdiv = gridDim.x / ups, gmod = gridDim.x - gdiv * ups;\n")
    << 
       "  const __amdgpu_buffer_rsrc_t RZ = __builtin_amdgcn_make_buffer_rsrc((void *)data, (short)0, 0, 0x00020000);\n"
       "  v4 la0[8], lb0[8];\n"
       "  {  // prologue: the first unit's leading positions of chunk 0\n"
       "  const u32 sbl = sb, uo = uu * 2048u + loff, uo1 = " << half << ";\n";
  rsrc_pair(o, "RD", "data", "ds", "stripe", s.k, "ub < ue");
  // Spec::dyn: per-stripe masks (skipped data positions, stored rows) from dm
  if (dyn) o << "  const u32 *DM = dm + (ub < ue ? stripe : 0ull) * dmw;\n";
  // (loads emitted below, once emit_loads exists)
  std::ostringstream hdr2;
  hdr2 << "#pragma unroll 1\n"
    << "  for (u64 u = ub; u < ue; u += step) {\n"
    << "  const bool stamp_on = blockIdx.x == 0u && u == ub + 2u * step;\n  STAMP(62u);\n"
    << 
       "  u32 sbl = sb;\n"
       "  asm volatile(\"\" : \"+s\"(sbl));  // shard offsets are recomputed per unit (SALU), not hoisted into VGPRs\n"
       "  const u32 uo = uu * 2048u + loff, uo1 = " << half << ";\n";
  rsrc_pair(hdr2, "RD", "data", "ds", "stripe", s.k, "");
  rsrc_pair(hdr2, "RO", "out", "os", "stripe", s.m, "");
  if (dyn) hdr2 << "  const u32 *DM = dm + stripe * dmw;\n";
  if (s.decode && dyn) hdr2 << "  const cptr DMc = (cptr)DM;\n";
  if (any_xor) rsrc_pair(hdr2, "RR", "rec", "rs", "stripe", s.m, "");
  hdr2 << "  u32 ";
  for (uint32_t r = 0; r < 8; r++)
    for (int i = 0; i < 8; i++) hdr2 << "w" << r << "_" << i << ", b" << r << "_" << i << ", c" << r << "_" << i << (r == 7 && i == 7 ? ";\n" : ", ");

  // LDS slot accesses: 4-dword accesses, planes 4q..4q+3 of a slot in quad q (dword
  // accesses measured 3.77 vs 3.54 ms on RS(200,55) in spite of 17 more VGPRs for the
  // 4-register tuples)
  auto lds_write = [&](const std::string &wexpr, uint32_t slot, const std::vector<std::string> &v) {
    // slot address = wexpr (runtime, in slots) + slot
    for (int q = 0; q < 2; q++)
      o << "  xch4[lq + " << wexpr << " * 128u + " << slot * 128 + q * 64 << "u] = (v4){" << v[4 * q] << ", "
        << v[4 * q + 1] << ", " << v[4 * q + 2] << ", " << v[4 * q + 3] << "};\n";
  };
  auto lds_read = [&](const std::string &wexpr, uint32_t slot, const std::vector<std::string> &v) {
    o << "  { const v4 q0 = xch4[lq + " << wexpr << " * 128u + " << slot * 128 << "u], q1 = xch4[lq + " << wexpr
      << " * 128u + " << slot * 128 + 64 << "u];\n";
    for (int i = 0; i < 4; i++) o << "  " << v[i] << " = q0[" << i << "]; " << v[4 + i] << " = q1[" << i << "];\n";
    o << "  }\n";
  };

  int nstamp = 0;  // STAMP ids (measurement builds)
  auto bar = [&]() {
    const std::string a = std::to_string(std::min(nstamp, 61)), b = std::to_string(std::min(nstamp + 1, 61));
    nstamp += 2;
    return "  STAMP(" + a + "u); BAR(); STAMP(" + b + "u);\n";
  };
  // ---- loads of chunk j (layout A: wave w reads positions w*8 + r), raw into la/lb
  std::vector<uint8_t> declared(P.truncs.size(), 0);
  auto emit_loads = [&](size_t j, uint32_t r0, uint32_t r1, const char *rd = "RD", const char *uo0 = "uo",
                        const char *uo1 = "uo1") {
    std::vector<uint32_t> vm(NW, 0);
    bool full = true;
    for (uint32_t w = 0; w < NW; w++)
      for (uint32_t r = 0; r < 8; r++) {
        if (P.valid[j][P.posA(w, r)]) vm[w] |= 1u << r;
        else full = false;
      }
    if (!declared[j]) o << "  v4 la" << j << "[8], lb" << j << "[8];\n";
    declared[j] = 1;
    if (r0 == r1) return vm;
    o << "  __builtin_amdgcn_sched_barrier(0);\n  {\n";
    if (!full) o << "  const u32 vm = " << mask_expr(vm) << ";\n";
    if (dyn)  // this wave's 8 positions of chunk j: one byte of the stripe's skip mask
      o << "  const u32 dsk = (" << (std::string(rd) == "RDn" ? "DMn" : "DM") << "[(" << j * C
        << "u + (w << 3)) >> 5] >> ((" << j * C << "u + (w << 3)) & 31u)) & 0xFFu;\n";
    for (uint32_t r = r0; r < r1; r++) {
      o << "  { const u32 so = (" << j * C + r << "u + (w << 3)) * sbl;\n    ";
      const std::string rd1 = std::string(rd) + "1";
      std::string cond = full ? "" : "((vm >> " + std::to_string(r) + ") & 1u)";
      if (dyn) cond = (cond.empty() ? "" : cond + " && ") + "!((dsk >> " + std::to_string(r) + ") & 1u)";
      const std::string rs = cond.empty() ? std::string(rd) : "(" + cond + " ? " + rd + " : RZ)";
      const std::string rs1 = cond.empty() ? rd1 : "(" + cond + " ? " + rd1 + " : RZ)";
      o << "la" << j << "[" << r << "] = LDB(" << rs << ", " << uo0 << ", so); lb" << j << "[" << r << "] = LDB(" << rs1
        << ", " << uo1 << ", so); }\n";
    }
    o << "  }\n  asm volatile(\"\" ::: \"memory\");\n  __builtin_amdgcn_sched_barrier(0);\n";
    return vm;
  };

  std::vector<uint8_t> acc_live(8, 0);  // layout B regs of the accumulator
  // RS_AMD_FFT_PREFETCH: positions of the next chunk loaded before this chunk's layers
  // (the rest just before their plane transform)
  const uint32_t pf = old_order ? 0u : static_cast<uint32_t>(prefetch_of(s));
  // the next unit's first pfu positions are loaded during this unit's FFT (encode) or
  // before its last data block (decode)
  const uint32_t pfu = pf;
  declared[0] = 1;  // la0 / lb0 live across units (cross-unit prefetch)
  std::vector<uint32_t> vm_next = emit_loads(0, 0, pfu);
  o << "  }\n" << hdr2.str();
  emit_loads(0, pfu, 8);
  for (size_t j = 0; j < P.truncs.size(); j++) {
    const std::vector<uint32_t> vm = vm_next;
    if (j > 0) emit_loads(j, pf, 8);
    o << "  // ---- chunk " << j << " (data shards " << j * C << "..): IFFT(size " << C << ", trunc " << P.truncs[j]
      << ", skew_delta " << (j + 1) * C << "), Generic.zig:80-147\n";
    // planes + basis change (shared code; invalid positions were read as zeros)
    g.ops = &g.st->ops_io;
    for (uint32_t r = 0; r < 8; r++) {
      bool any = false;
      for (uint32_t w = 0; w < NW; w++) any |= (vm[w] >> r & 1) != 0;
      if (!any) continue;
      o << "  { u32 Q[8]; planes2(la" << j << "[" << r << "], lb" << j << "[" << r << "], Q, KM);\n";
      for (int i = 0; i < 8; i++) o << "  w" << r << "_" << i << " = Q[" << i << "];\n";
      g.op(4 + 48);
      const auto W = Gen::regs(wname(r));
      g.basis_change(W);
      o << "  }\n";
    }
    if (j + 1 < P.truncs.size()) vm_next = emit_loads(j + 1, 0, pf);  // in flight during this chunk's layers
    // ---- layout A layers (bits 0..2), specialised per wave; liveness first
    std::vector<std::vector<uint8_t>> liveA(NW, std::vector<uint8_t>(8, 0));
    for (uint32_t w = 0; w < NW; w++) {
      bool z[8];
      for (uint32_t r = 0; r < 8; r++) z[r] = !(vm[w] >> r & 1);
      for (const Layer &L : P.ifft[j]) {
        if (!P.inA(L.bit)) continue;
        for (const Bf &b : L.bf)
          if (P.waveA(b.x) == w && !(z[P.regA(b.x)] && z[P.regA(b.y)])) z[P.regA(b.x)] = z[P.regA(b.y)] = false;
      }
      for (uint32_t r = 0; r < 8; r++) liveA[w][r] = !z[r];
    }
    std::vector<uint8_t> liveB(8, 0);
    for (uint32_t w = 0; w < NW; w++)
      for (uint32_t r = 0; r < 8; r++)
        if (liveA[w][r]) liveB[P.regB(P.posA(w, r))] = 1;
    // A layers, then A -> B through LDS: A wave a writes reg r (position p) to slot
    // (p & (NW-1)) * 8 + (p >> WB); the slots are free (every wave passed the barrier
    // after the previous exchange's reads)
    g.ops = &g.st->ops_a;
    o << "  {\n  LQ();\n";
    for (uint32_t w = 0; w < NW; w++) {
      bool z[8];
      for (uint32_t r = 0; r < 8; r++) z[r] = !(vm[w] >> r & 1);
      o << "  " << (w ? "else if" : "if") << " (w == " << w << "u) {\n";
      for (const Layer &L : P.ifft[j]) {
        if (!P.inA(L.bit)) continue;
        for (const Bf &b : L.bf) {
          if (P.waveA(b.x) != w) continue;
          const uint32_t rx = P.regA(b.x), ry = P.regA(b.y);
          g.butterfly(wname(rx), z[rx], wname(ry), z[ry], true, P.get_tw(b.log_m));
        }
      }
      for (uint32_t r = 0; r < 8; r++) {
        const uint32_t p = P.posA(w, r), t = P.regB(p);
        if (!liveB[t]) continue;
        const uint32_t slot = P.waveB(p) * 8 + t;
        std::vector<std::string> v = Gen::regs(wname(r));
        if (z[r]) v.assign(8, "0u");
        lds_write("0", slot, v);
      }
      o << "  }\n";
    }
    o << bar();
    bool zb[8];
    for (uint32_t t = 0; t < 8; t++) {
      zb[t] = !liveB[t];
      if (!liveB[t]) continue;
      lds_read("(w * 8u)", t, Gen::regs(bname(t)));
    }
    o << bar() << "  }\n";  // every wave has read its slots: the next exchange may write
    // ---- layout B layers (bits >= 3), one code path for all waves
    g.ops = &g.st->ops_b;
    for (const Layer &L : P.ifft[j]) {
      if (P.inA(L.bit)) continue;
      for (const Bf &b : L.bf) {
        if (P.waveB(b.x) != 0) continue;  // twiddles are uniform over the wave bits
        const uint32_t tx = P.regB(b.x), ty = P.regB(b.y);
        g.butterfly(bname(tx), zb[tx], bname(ty), zb[ty], true, P.get_tw(b.log_m));
      }
    }
    // XOR-fold into the accumulator, root.zig:150-166
    for (uint32_t t = 0; t < 8; t++) {
      if (zb[t]) continue;
      if (acc_live[t])
        g.xor_into(Gen::regs(cname(t)), Gen::regs(bname(t)));
      else
        g.copy(Gen::regs(cname(t)), Gen::regs(bname(t)));
      acc_live[t] = 1;
    }
    for (uint32_t t = 0; t < 8; t++)
      if (acc_live[t]) g.pin(Gen::regs(cname(t)));
    o << "  __builtin_amdgcn_sched_barrier(0);\n  asm volatile(\"\" ::: \"memory\");\n";
  }

  // ---- FFT(size C, trunc m, skew_delta 0), Generic.zig:15-78 — needed positions first
  std::vector<uint8_t> need(C, 0);  // at the start of the A layers
  {
    std::vector<uint8_t> nd(C, 0);
    for (uint32_t q = 0; q < C; q++) nd[q] = P.out_mode[q] != kOutNone;
    for (auto it = P.fft.rbegin(); it != P.fft.rend(); ++it) {
      if (!P.inA(it->bit)) continue;
      for (const Bf &b : it->bf)
        if (nd[b.x] || nd[b.y]) nd[b.x] = nd[b.y] = 1;
    }
    need = nd;
  }
  // decode: the recovery rows R of this wave's 8 positions (layout A), in flight during the
  // FFT's B layers, its exchange and its A layers
  const uint32_t dwm = dyn_store_word(P) + 2;
  auto emit_rec_loads = [&]() {
    o << "  const u32 ub0 = DMc[" << dwm + 1 << "], ub1 = DMc[" << dwm + 2 << "];\n";
    for (uint32_t r = 0; r < 8; r++)
      o << "  const u32 pd" << r << " = w * 8u + " << r << "u;\n  const bool us" << r << " = ((pd" << r
        << " < 32u ? ub0 >> pd" << r << " : ub1 >> (pd" << r << " - 32u)) & 1u) != 0u;\n  const v4 ra" << r
        << " = LDB(us" << r << " ? RR : RZ, uo, pd" << r << " * sbl), rb" << r << " = LDB(us" << r
        << " ? RR1 : RZ, uo1, pd" << r << " * sbl);\n";
  };
  // Spec::present: a wave's rows of R (static), loaded where RS_AMD_PDEC_RLOAD says; r0..r1 of them
  const int rload = spat ? ((dbg & 32) ? 2 : rload_of()) : 0;
  auto emit_rows_R = [&](uint32_t w, uint32_t r0, uint32_t r1) {
    for (uint32_t r = r0; r < r1; r++) {
      const uint32_t p = P.posA(w, r);
      if (p < s.m && inR[p])
        o << "  ra" << r << " = LDB(RR, uo, " << p << "u * sbl); rb" << r << " = LDB(RR1, uo1, " << p << "u * sbl);\n";
    }
  };
  if (tail && rload) {
    o << "  v4 ";
    for (uint32_t r = 0; r < 8; r++) o << "ra" << r << ", rb" << r << (r < 7 ? ", " : ";\n");
  }
  if (tail && rload == 2) {  // before the final FFT's B layers (round 4 measured: spills)
    bool firstw = true;
    for (uint32_t w = 0; w < NW; w++) {
      bool any = false;
      for (uint32_t r = 0; r < 8; r++) any |= P.posA(w, r) < s.m && inR[P.posA(w, r)];
      if (!any) continue;
      o << "  " << (firstw ? "if" : "else if") << " (w == " << w << "u) {\n";
      firstw = false;
      emit_rows_R(w, 0, 8);
      o << "  }\n";
    }
  } else if (tail && !old_order && !spat) {
    emit_rec_loads();
  }
  o << "  // ---- FFT(size " << C << ", trunc " << s.m << ", skew_delta 0), Generic.zig:15-78\n";
  g.ops = &g.st->ops_b;
  bool zc[8];
  for (uint32_t t = 0; t < 8; t++) zc[t] = !acc_live[t];
  for (const Layer &L : P.fft) {
    if (P.inA(L.bit)) continue;
    for (const Bf &b : L.bf) {
      if (P.waveB(b.x) != 0) continue;
      const uint32_t tx = P.regB(b.x), ty = P.regB(b.y);
      g.butterfly(cname(tx), zc[tx], cname(ty), zc[ty], false, P.get_tw(b.log_m));
    }
  }
  // the next unit's leading chunk-0 positions, in flight during this unit's last exchange and stores
  o << "  u64 stripe_n = stripe + gdiv;\n  u32 uu_n = uu + gmod;\n  if (uu_n >= ups) { uu_n -= ups; stripe_n++; }\n";
  auto emit_next_unit_loads = [&]() {
    o << "  {\n  const u32 uon = uu_n * 2048u + loff, uon1 = " << (two ? "loff" : "uon + 1024u") << ";\n";
    rsrc_pair(o, "RDn", "data", "ds", "stripe_n", s.k, "u + step < ue");
    if (dyn) o << "  const u32 *DMn = dm + ((u + step < ue) ? stripe_n : 0ull) * dmw;\n";
    emit_loads(0, 0, pfu, "RDn", "uon", "uon1");
    o << "  }\n";
  };
  if (pfu && !s.decode) emit_next_unit_loads();
  // B -> A: B wave w writes reg t (position p = t << WB | w) to slot p; then every
  // wave reads its 8 slots (shared code) and passes a barrier before the
  // specialised A layers, so the next unit's first exchange may write at once
  std::vector<uint8_t> needB(8, 0);
  for (uint32_t q = 0; q < C; q++)
    if (need[q]) needB[P.regB(q)] = 1;
  std::vector<uint8_t> readA(8, 0);
  for (uint32_t q = 0; q < C; q++)
    if (need[q] && !zc[P.regB(q)]) readA[P.regA(q)] = 1;
  o << "  {\n  LQ();\n";
  for (uint32_t t = 0; t < 8; t++) {
    if (!needB[t] || zc[t]) continue;
    lds_write("w", t << P.WB, Gen::regs(cname(t)));
  }
  o << bar();
  for (uint32_t r = 0; r < 8; r++) {
    if (!readA[r]) continue;
    lds_read("(w * 8u)", r, Gen::regs(wname(r)));
  }
  o << bar() << "  }\n";
  g.ops = &g.st->ops_a;
  auto anyout_of = [&](uint32_t w) {
    bool anyout = false;
    for (uint32_t r = 0; r < 8; r++) anyout |= P.out_mode[P.posA(w, r)] != kOutNone;
    return anyout;
  };
  // a wave's A layers of the final FFT; the decode kernels keep Enc(d') rows p < m in registers
  // for the tail (Spec::present: emitted inside the tail's per-wave branch, below, with the
  // wave's rows of R in flight during them when RS_AMD_PDEC_RLOAD is 1 or 3)
  auto final_A = [&](uint32_t w, std::vector<uint8_t> &zout) {
    if (tail && (rload == 1 || rload == 3)) {  // this wave's rows of R, in flight during its A layers
      emit_rows_R(w, 0, rload == 1 ? 8 : 4);
      o << "  asm volatile(\"\" ::: \"memory\");\n  __builtin_amdgcn_sched_barrier(0);\n";
    }
    g.ops = &g.st->ops_a;
    bool z[8];
    for (uint32_t r = 0; r < 8; r++) {
      const uint32_t p = P.posA(w, r);
      z[r] = zc[P.regB(p)] || !need[p];
    }
    for (const Layer &L : P.fft) {
      if (!P.inA(L.bit)) continue;
      for (const Bf &b : L.bf) {
        if (P.waveA(b.x) != w) continue;
        const uint32_t rx = P.regA(b.x), ry = P.regA(b.y);
        g.butterfly(wname(rx), z[rx], wname(ry), z[ry], false, P.get_tw(b.log_m));
      }
    }
    zout.assign(z, z + 8);
    if (s.decode)
      for (uint32_t r = 0; r < 8; r++)
        if (P.posA(w, r) < s.m && z[r])
          for (int i = 0; i < 8; i++) o << "  " << wname(r) << "_" << i << " = 0u;\n";
  };
  bool first = true;
  for (uint32_t w = 0; w < NW && !(spat && tail); w++) {
    if (!anyout_of(w)) continue;
    o << "  " << (first ? "if" : "else if") << " (w == " << w << "u) {\n";
    first = false;
    std::vector<uint8_t> zv;
    final_A(w, zv);
    bool z[8];
    for (uint32_t r = 0; r < 8; r++) z[r] = zv[r] != 0;
    if (s.decode) {
      o << "  }\n";
      continue;
    }
    // basis change back, planes -> bytes, store (or rec ^ parity)
    g.ops = &g.st->ops_io;
    if (dyn)  // rows this stripe stores: one byte of its store mask
      o << "  const u32 dst = (DM[" << dyn_store_word(P) + w / 4 << "u] >> " << (w % 4) * 8 << ") & 0xFFu;\n";
    for (uint32_t r = 0; r < 8; r++) {
      const uint32_t p = P.posA(w, r);
      if (P.out_mode[p] == kOutNone) continue;
      const auto W = Gen::regs(wname(r));
      if (z[r])
        for (int i = 0; i < 8; i++) o << "  " << W[i] << " = 0u;\n";
      else
        g.basis_change(W);
      o << "  { u32 Q[8] = {";
      for (int i = 0; i < 8; i++) o << W[i] << (i < 7 ? ", " : "};\n");
      o << "    v4 a, b; unplanes2(Q, a, b, KM);\n";
      g.op(4 + 48);
      o << "    const u32 so = " << p << "u * sbl;\n";
      if (P.out_mode[p] == kOutXorRec) o << "    a ^= LDB(RR, uo, so); b ^= LDB(RR1, uo1, so);\n";
      if (dyn)
        o << "    const bool keep = (dst >> " << r << ") & 1u;\n    STB(a, keep ? RO : RZ, uo, so); STB(b, keep ? RO1 : RZ, uo1, so); }\n";
      else
        o << "    STB(a, RO, uo, so); STB(b, RO1, uo1, so); }\n";
    }
    g.ops = &g.st->ops_a;
    o << "  }\n";
  }
  if (s.decode && !tail) {  // measurement build: Enc(d') only, kept live
    for (uint32_t r = 0; r < 8; r++) {
      o << "  asm volatile(\"\" ::";
      for (int i = 0; i < 8; i++) o << (i ? ", " : " ") << "\"v\"(" << wname(r) << "_" << i << ")";
      o << ");\n";
    }
    if (pfu) emit_next_unit_loads();
  }
  if (tail && spat) {
    // ---- decode tail, pattern compiled in (Spec::present): as below, with the locator
    // scalars as constant multiplies and every row, block and output static
    auto cmul = [&](const std::vector<std::string> &X, uint32_t lg) {  // X *= exp[lg] in place
      std::vector<std::string> Y(8);
      o << "  __builtin_amdgcn_sched_barrier(0);\n  {\n  u32 ";
      for (int i = 0; i < 8; i++) {
        Y[i] = g.fresh("zy");
        o << Y[i] << (i < 7 ? ", " : ";\n");
      }
      g.mul(Y, false, X, twiddle(static_cast<uint16_t>(lg), false));
      for (int i = 0; i < 8; i++) o << "  " << X[i] << " = " << Y[i] << ";\n";
      o << "  }\n";
    };
    const std::vector<Layer> il = ifft_layers(C, s.m, 0);
    std::vector<uint8_t> liveB(8, 0);
    std::vector<std::vector<uint8_t>> z0(NW, std::vector<uint8_t>(8, 1));  // zero at the IFFT's start
    for (uint32_t w = 0; w < NW; w++) {
      bool z[8];
      for (uint32_t r = 0; r < 8; r++) z[r] = z0[w][r] = !(P.posA(w, r) < s.m && inR[P.posA(w, r)]);
      for (const Layer &L : il) {
        if (!P.inA(L.bit)) continue;
        for (const Bf &b : L.bf)
          if (P.waveA(b.x) == w && !(z[P.regA(b.x)] && z[P.regA(b.y)])) z[P.regA(b.x)] = z[P.regA(b.y)] = false;
      }
      for (uint32_t r = 0; r < 8; r++)
        if (!z[r]) liveB[P.regB(P.posA(w, r))] = 1;
    }
    // (the final FFT's A layers), syndromes times L_p, IFFT A layers (per wave), A -> B
    o << "  {\n  LQ();\n";
    for (uint32_t w = 0; w < NW; w++) {
      o << "  " << (w ? "else if" : "if") << " (w == " << w << "u) {\n";
      if (anyout_of(w)) {
        std::vector<uint8_t> zv;
        final_A(w, zv);
        o << "  __builtin_amdgcn_sched_barrier(0);\n";
      }
      if (!rload)  // this wave's rows of R, in flight together
        for (uint32_t r = 0; r < 8; r++)
          if (!z0[w][r])
            o << "  const v4 ra" << r << " = LDB(RR, uo, " << P.posA(w, r) << "u * sbl), rb" << r << " = LDB(RR1, uo1, "
              << P.posA(w, r) << "u * sbl);\n";
      if (rload == 3) emit_rows_R(w, 4, 8);
      bool z[8];
      for (uint32_t r = 0; r < 8; r++) {
        z[r] = z0[w][r];
        if (z[r]) continue;
        const uint32_t p = P.posA(w, r);
        const auto W = Gen::regs(wname(r));
        g.ops = &g.st->ops_io;
        o << "  __builtin_amdgcn_sched_barrier(0);\n  { u32 Q[8]; planes2(ra" << r << ", rb" << r << ", Q, KM);\n";
        std::vector<std::string> q(8);
        for (int i = 0; i < 8; i++) q[i] = "Q[" + std::to_string(i) + "]";
        g.basis_change(q);
        for (int i = 0; i < 8; i++) o << "  " << W[i] << " ^= Q[" << i << "];\n";
        o << "  }\n";
        cmul(W, lp_log[p]);
      }
      g.ops = &g.st->ops_a;
      for (const Layer &L : il) {
        if (!P.inA(L.bit)) continue;
        for (const Bf &b : L.bf) {
          if (P.waveA(b.x) != w) continue;
          const uint32_t rx = P.regA(b.x), ry = P.regA(b.y);
          g.butterfly(wname(rx), z[rx], wname(ry), z[ry], true, P.get_tw(b.log_m));
        }
      }
      for (uint32_t r = 0; r < 8; r++) {
        const uint32_t p = P.posA(w, r), t = P.regB(p);
        if (!liveB[t]) continue;
        std::vector<std::string> v = Gen::regs(wname(r));
        if (z[r]) v.assign(8, "0u");
        lds_write("0", P.waveB(p) * 8 + t, v);
      }
      o << "  }\n";
    }
    o << bar();
    bool za[8];
    for (uint32_t t = 0; t < 8; t++) {
      za[t] = !liveB[t];
      if (liveB[t]) lds_read("(w * 8u)", t, Gen::regs(cname(t)));
    }
    o << bar() << "  }\n";
    g.ops = &g.st->ops_b;
    for (const Layer &L : il) {
      if (P.inA(L.bit)) continue;
      for (const Bf &b : L.bf) {
        if (P.waveB(b.x) != 0) continue;
        const uint32_t tx = P.regB(b.x), ty = P.regB(b.y);
        g.butterfly(cname(tx), za[tx], cname(ty), za[ty], true, P.get_tw(b.log_m));
      }
    }
    for (uint32_t t = 0; t < 8; t++)
      if (!za[t]) g.pin(Gen::regs(cname(t)));
    // per data block K with an erasure: FFT(size C, trunc t_K, skew KC) of a, pruned to
    // the butterflies an erased shard's evaluation needs
    const uint32_t nblk = (s.k + C - 1) / C;
    uint32_t last_blk = 0;
    for (uint32_t K = 1; K <= nblk; K++)
      for (uint32_t g0 = (K - 1) * C; g0 < std::min<uint32_t>(s.k, K * C); g0++)
        if (!s.present[g0]) last_blk = K;
    if (!last_blk && pfu) emit_next_unit_loads();
    for (uint32_t K = 1; K <= last_blk; K++) {
      const uint32_t tK = std::min<uint32_t>(C, s.k - (K - 1) * C), g0 = (K - 1) * C;
      bool anyK = false;
      for (uint32_t q = 0; q < tK; q++) anyK |= !s.present[g0 + q];
      if (!anyK) continue;
      const std::vector<Layer> fl = fft_layers(C, tK, static_cast<uint64_t>(K) * C);
      // backward: positions needed (A layers), then register rows needed (B layers)
      std::vector<uint8_t> need(C, 0);
      for (uint32_t q = 0; q < tK; q++) need[q] = !s.present[g0 + q];
      std::map<std::pair<size_t, size_t>, bool> emit;  // (layer, butterfly) -> emitted
      for (size_t li = fl.size(); li-- > 0;) {
        if (!P.inA(fl[li].bit)) continue;
        for (size_t bi = fl[li].bf.size(); bi-- > 0;) {
          const Bf &b = fl[li].bf[bi];
          const bool e = need[b.x] || need[b.y];
          emit[{li, bi}] = e;
          if (e) need[b.x] = need[b.y] = 1;
        }
      }
      std::vector<uint8_t> nB(8, 0);  // rows the B phase must deliver
      for (uint32_t q = 0; q < C; q++)
        if (need[q]) nB[P.regB(q)] = 1;
      std::vector<uint8_t> nb = nB;
      for (size_t li = fl.size(); li-- > 0;) {
        if (P.inA(fl[li].bit)) continue;
        for (size_t bi = fl[li].bf.size(); bi-- > 0;) {
          const Bf &b = fl[li].bf[bi];
          if (P.waveB(b.x) != 0) continue;
          const uint32_t tx = P.regB(b.x), ty = P.regB(b.y);
          const bool e = nb[tx] || nb[ty];
          emit[{li, bi}] = e;
          if (e) nb[tx] = nb[ty] = 1;
        }
      }
      const bool last = K == last_blk;
      auto bn = [&](uint32_t t) { return last ? cname(t) : bname(t); };
      if (last && pfu) emit_next_unit_loads();
      o << "  __builtin_amdgcn_sched_barrier(0);\n  {  // data block " << K << ": FFT(size " << C << ", trunc " << tK
        << ", skew_delta " << K * C << ")\n";
      g.ops = &g.st->ops_b;
      bool zb[8];
      for (uint32_t t = 0; t < 8; t++) {
        zb[t] = za[t] || !nb[t];
        if (!zb[t] && !last) g.copy(Gen::regs(bname(t)), Gen::regs(cname(t)));
      }
      for (size_t li = 0; li < fl.size(); li++) {
        if (P.inA(fl[li].bit)) continue;
        for (size_t bi = 0; bi < fl[li].bf.size(); bi++) {
          const Bf &b = fl[li].bf[bi];
          if (P.waveB(b.x) != 0 || !emit[{li, bi}]) continue;
          const uint32_t tx = P.regB(b.x), ty = P.regB(b.y);
          g.butterfly(bn(tx), zb[tx], bn(ty), zb[ty], false, P.get_tw(b.log_m));
        }
      }
      std::vector<uint8_t> rA(8, 0);
      for (uint32_t q = 0; q < C; q++)
        if (need[q] && !zb[P.regB(q)]) rA[P.regA(q)] = 1;
      o << "  {\n  LQ();\n";
      for (uint32_t t = 0; t < 8; t++)
        if (nB[t] && !zb[t]) lds_write("w", t << P.WB, Gen::regs(bn(t)));
      o << bar();
      for (uint32_t r = 0; r < 8; r++)
        if (rA[r]) lds_read("(w * 8u)", r, Gen::regs(wname(r)));
      o << bar() << "  }\n";
      // A layers and the erased shards' outputs, per wave
      bool firstw = true;
      for (uint32_t w = 0; w < NW; w++) {
        bool anyw = false;
        for (uint32_t r = 0; r < 8; r++) {
          const uint32_t q = P.posA(w, r);
          anyw |= q < tK && !s.present[g0 + q];
        }
        if (!anyw) continue;
        o << "  " << (firstw ? "if" : "else if") << " (w == " << w << "u) {\n";
        firstw = false;
        g.ops = &g.st->ops_a;
        bool z[8];
        for (uint32_t r = 0; r < 8; r++) z[r] = zb[P.regB(P.posA(w, r))] || !need[P.posA(w, r)];
        for (size_t li = 0; li < fl.size(); li++) {
          if (!P.inA(fl[li].bit)) continue;
          for (size_t bi = 0; bi < fl[li].bf.size(); bi++) {
            const Bf &b = fl[li].bf[bi];
            if (P.waveA(b.x) != w || !emit[{li, bi}]) continue;
            const uint32_t rx = P.regA(b.x), ry = P.regA(b.y);
            g.butterfly(wname(rx), z[rx], wname(ry), z[ry], false, P.get_tw(b.log_m));
          }
        }
        g.ops = &g.st->ops_io;
        for (uint32_t r = 0; r < 8; r++) {
          const uint32_t q = P.posA(w, r), gi = g0 + q;
          if (q >= tK || s.present[gi]) continue;
          const auto W = Gen::regs(wname(r));
          if (z[r] || cg_log[gi] > kModulus) {
            for (int i = 0; i < 8; i++) o << "  " << W[i] << " = 0u;\n";
          } else {
            cmul(W, cg_log[gi]);
            g.basis_change(W);
          }
          o << "  __builtin_amdgcn_sched_barrier(0);\n  { u32 X[8] = {";
          for (int i = 0; i < 8; i++) o << W[i] << (i < 7 ? ", " : "};\n");
          o << "  v4 a, b; unplanes2(X, a, b, KM);\n  STB(a, RO, uo, " << out_row[gi] << "u * sbl); STB(b, RO1, uo1, "
            << out_row[gi] << "u * sbl); }\n";
        }
        o << "  }\n";
      }
      o << "  }\n";
    }
  } else if (tail) {
    // ---- decode tail (Spec::decode): w_p = L_p (rec_p ^ Enc_p) for the
    // rows R (layout A), a = IFFT(size C, trunc m, skew 0) (A then B), and per data block K
    // with an erasure: FFT(a, size C, trunc t_K, skew KC) (B then A), x_g = (L'_g beta_K) y_q
    const uint32_t mko = decode_mask_offset(s);
    g.ops = &g.st->ops_io;
    o << "  {  // syndromes of the rows R times the locator (one code path, runtime scalars)\n";
    if (old_order) emit_rec_loads();
    for (uint32_t r = 0; r < 8; r++) {
      const auto W = Gen::regs(wname(r));
      o << "  if (us" << r << ") {\n  u32 Q[8]; planes2(ra" << r << ", rb" << r << ", Q, KM);\n";
      std::vector<std::string> q(8);
      for (int i = 0; i < 8; i++) q[i] = "Q[" + std::to_string(i) + "]";
      g.basis_change(q);
      o << "  u32 X[8] = {";
      for (int i = 0; i < 8; i++) o << W[i] << " ^ Q[" << i << "]" << (i < 7 ? ", " : "};\n");
      o << "  rmul(X, (cptr)(DM + " << mko << "u + pd" << r << " * 128u), KM);\n";
      for (int i = 0; i < 8; i++) o << "  " << W[i] << " = X[" << i << "];\n";
      o << "  } else {\n";
      for (int i = 0; i < 8; i++) o << "  " << W[i] << " = 0u;\n";
      o << "  }\n";
    }
    o << "  }\n";
    // IFFT(size C, trunc m, skew 0): A layers per wave, A -> B, B layers
    const std::vector<Layer> il = ifft_layers(C, s.m, 0);
    std::vector<std::vector<uint8_t>> zA(NW, std::vector<uint8_t>(8, 0));
    std::vector<uint8_t> liveB(8, 0);
    for (uint32_t w = 0; w < NW; w++) {
      bool z[8];
      for (uint32_t r = 0; r < 8; r++) z[r] = P.posA(w, r) >= s.m;
      for (const Layer &L : il) {
        if (!P.inA(L.bit)) continue;
        for (const Bf &b : L.bf)
          if (P.waveA(b.x) == w && !(z[P.regA(b.x)] && z[P.regA(b.y)])) z[P.regA(b.x)] = z[P.regA(b.y)] = false;
      }
      for (uint32_t r = 0; r < 8; r++) {
        zA[w][r] = z[r];
        if (!z[r]) liveB[P.regB(P.posA(w, r))] = 1;
      }
    }
    g.ops = &g.st->ops_a;
    o << "  {\n  LQ();\n";
    for (uint32_t w = 0; w < NW; w++) {
      bool z[8];
      for (uint32_t r = 0; r < 8; r++) z[r] = P.posA(w, r) >= s.m;
      o << "  " << (w ? "else if" : "if") << " (w == " << w << "u) {\n";
      for (const Layer &L : il) {
        if (!P.inA(L.bit)) continue;
        for (const Bf &b : L.bf) {
          if (P.waveA(b.x) != w) continue;
          const uint32_t rx = P.regA(b.x), ry = P.regA(b.y);
          g.butterfly(wname(rx), z[rx], wname(ry), z[ry], true, P.get_tw(b.log_m));
        }
      }
      for (uint32_t r = 0; r < 8; r++) {
        const uint32_t p = P.posA(w, r), t = P.regB(p);
        if (!liveB[t]) continue;
        std::vector<std::string> v = Gen::regs(wname(r));
        if (z[r]) v.assign(8, "0u");
        lds_write("0", P.waveB(p) * 8 + t, v);
      }
      o << "  }\n";
    }
    o << bar();
    bool za[8];
    for (uint32_t t = 0; t < 8; t++) {
      za[t] = !liveB[t];
      if (liveB[t]) lds_read("(w * 8u)", t, Gen::regs(cname(t)));
    }
    o << bar() << "  }\n";
    g.ops = &g.st->ops_b;
    for (const Layer &L : il) {
      if (P.inA(L.bit)) continue;
      for (const Bf &b : L.bf) {
        if (P.waveB(b.x) != 0) continue;
        const uint32_t tx = P.regB(b.x), ty = P.regB(b.y);
        g.butterfly(cname(tx), za[tx], cname(ty), za[ty], true, P.get_tw(b.log_m));
      }
    }
    for (uint32_t t = 0; t < 8; t++)
      if (!za[t]) g.pin(Gen::regs(cname(t)));
    // per data block K: FFT(size C, trunc t_K, skew KC) of a
    const uint32_t nblk = (s.k + C - 1) / C;
    for (uint32_t K = 1; K <= nblk; K++) {
      const uint32_t tK = std::min<uint32_t>(C, s.k - (K - 1) * C);
      const std::vector<Layer> fl = fft_layers(C, tK, static_cast<uint64_t>(K) * C);
      std::vector<uint8_t> nd(C, 0);
      for (uint32_t q = 0; q < tK; q++) nd[q] = 1;
      for (auto it = fl.rbegin(); it != fl.rend(); ++it) {
        if (!P.inA(it->bit)) continue;
        for (const Bf &b : it->bf)
          if (nd[b.x] || nd[b.y]) nd[b.x] = nd[b.y] = 1;
      }
      // the last block transforms a in place (its last use), and the next unit's leading
      // positions are loaded before it (a's registers free up there)
      const bool last = K == nblk && !old_order;
      auto bn = [&](uint32_t t) { return last ? cname(t) : bname(t); };
      if (last && pfu) emit_next_unit_loads();
      o << "  __builtin_amdgcn_sched_barrier(0);\n  if ((DMc[" << dwm << "] >> " << K << "u) & 1u) {  // data block " << K
        << ": FFT(size " << C << ", trunc " << tK << ", skew_delta " << K * C << ")\n";
      g.ops = &g.st->ops_b;
      bool zb[8];
      for (uint32_t t = 0; t < 8; t++) {
        zb[t] = za[t];
        if (!za[t] && !last) g.copy(Gen::regs(bname(t)), Gen::regs(cname(t)));
      }
      for (const Layer &L : fl) {
        if (P.inA(L.bit)) continue;
        for (const Bf &b : L.bf) {
          if (P.waveB(b.x) != 0) continue;
          const uint32_t tx = P.regB(b.x), ty = P.regB(b.y);
          g.butterfly(bn(tx), zb[tx], bn(ty), zb[ty], false, P.get_tw(b.log_m));
        }
      }
      std::vector<uint8_t> nB(8, 0), rA(8, 0);
      for (uint32_t q = 0; q < C; q++)
        if (nd[q]) {
          nB[P.regB(q)] = 1;
          if (!zb[P.regB(q)]) rA[P.regA(q)] = 1;
        }
      o << "  {\n  LQ();\n";
      for (uint32_t t = 0; t < 8; t++)
        if (nB[t] && !zb[t]) lds_write("w", t << P.WB, Gen::regs(bn(t)));
      o << bar();
      for (uint32_t r = 0; r < 8; r++)
        if (rA[r]) lds_read("(w * 8u)", r, Gen::regs(wname(r)));
      o << bar() << "  }\n";
      g.ops = &g.st->ops_a;
      bool firstw = true;
      for (uint32_t w = 0; w < NW; w++) {
        if (P.posA(w, 0) >= tK) continue;
        // a wave whose 8 shards of the block are all received skips its layers (per-stripe
        // patterns spread few losses over many blocks)
        const uint32_t g0 = (K - 1) * C + 8 * w;
        o << "  " << (firstw ? "if" : "else if") << " (w == " << w << "u) {\n  if ((DMc[" << g0 / 32 << "] >> "
          << g0 % 32 << "u) & 0xFFu) {\n";
        firstw = false;
        bool z[8];
        for (uint32_t r = 0; r < 8; r++) {
          const uint32_t p = P.posA(w, r);
          z[r] = zb[P.regB(p)] || !nd[p];
        }
        for (const Layer &L : fl) {
          if (!P.inA(L.bit)) continue;
          for (const Bf &b : L.bf) {
            if (P.waveA(b.x) != w) continue;
            const uint32_t rx = P.regA(b.x), ry = P.regA(b.y);
            g.butterfly(wname(rx), z[rx], wname(ry), z[ry], false, P.get_tw(b.log_m));
          }
        }
        for (uint32_t r = 0; r < 8; r++)
          if (P.posA(w, r) < tK && z[r])
            for (int i = 0; i < 8; i++) o << "  " << wname(r) << "_" << i << " = 0u;\n";
        o << "  }\n  }\n";
      }
      // erased shards of the block: x_g = (L'_g beta_K) y_q, one code path for all waves
      g.ops = &g.st->ops_io;
      for (uint32_t r = 0; r < 8; r++) {
        const auto W = Gen::regs(wname(r));
        const uint32_t g0 = (K - 1) * C;
        o << "  { const u32 q = w * 8u + " << r << "u;\n  const u32 row = q < " << tK << "u ? DMc[" << dwm + 3 + g0
          << "u + q] : 0xFFFFFFFFu;\n  if (row != 0xFFFFFFFFu) {\n  u32 X[8] = {";
        for (int i = 0; i < 8; i++) o << W[i] << (i < 7 ? ", " : "};\n");
        o << "  rmul(X, (cptr)(DM + " << mko + 128 * (s.m + g0) << "u + q * 128u), KM);\n";
        std::vector<std::string> xs(8);
        for (int i = 0; i < 8; i++) xs[i] = "X[" + std::to_string(i) + "]";
        g.basis_change(xs);
        o << "  v4 a, b; unplanes2(X, a, b, KM);\n  const u32 so = row * sbl;\n  STB(a, RO, uo, so); STB(b, RO1, uo1, so);\n"
          << "  }\n  }\n";
      }
      o << "  }\n";
    }
  }
  o << "  STAMP(63u);\n  stripe = stripe_n; uu = uu_n;\n";
  o << "  }\n}\n";
  return o.str();
}

}  // namespace

bool supports(uint64_t k, uint64_t m, uint64_t shard_bytes, bool chunk16) {
  // chunk 16 (9 <= m <= 16, two waves per workgroup): the per-stripe pattern path's
  // syndromes (chunk16); encodes keep those codes on the networks (no faster there,
  // DESIGN.md §3.5)
  const uint64_t m_min = chunk16 ? 9 : 17;
  if (!basis().ok || m < m_min || m > 64 || k == 0) return false;
  const uint64_t C = ceil_pow2(m);
  if (C != 16 && C != 32 && C != 64) return false;
  // high rate (root.zig:397-415) with this chunk
  const uint64_t pk = ceil_pow2(k);
  if (!(pk > C || (pk == C && k <= m))) return false;
  if ((k + C - 1) / C > kMaxChunks) return false;
  if (shard_bytes != 1024 && (shard_bytes == 0 || shard_bytes % kUnitBytes)) return false;
  return k * shard_bytes + 4096 < 0x80000000ull && m * shard_bytes + 4096 < 0x80000000ull;
}

uint32_t pieces(uint64_t shard_bytes) { return shard_bytes == 1024 ? 2u : 1u; }

bool supports_inverse(uint64_t k, uint64_t m, uint64_t shard_bytes) {
  return k == m && ceil_pow2(m) == m && supports(k, m, shard_bytes);
}

std::string cache_key(const Spec &s) {
  // code-shape knobs are part of the key (read when the source is generated)
  std::string k = "fft4:p" + std::to_string(prefetch_of(s)) + (s.decode && !s.present.empty() && rload_of() ? ":rl" + std::to_string(rload_of()) : "") + ":s" + std::to_string(sched_of()) + ":d" +
                  std::to_string(debug_of()) + ":g" + std::to_string(rmul_group()) + ":k" + std::to_string(vmask_of()) + ":" +
                  std::to_string(s.k) + ":" +
                  std::to_string(s.m) + ":" + std::to_string(s.flags) + ":" +
                  (s.pieces > 1 ? "p" + std::to_string(s.pieces) + ":" : "") + (s.inverse ? "inv:" : "") +
                  (s.dyn ? "dyn:" : "") + (s.decode ? "dec:" : "") + (s.blocked ? "blk:" : "");
  if (!s.present.empty()) {
    k += "pat:";
    for (uint8_t b : s.present) k.push_back(b ? '1' : '0');
  }
  for (uint8_t b : s.skip) k.push_back(static_cast<char>('0' + b));
  k.push_back(':');
  for (uint8_t b : s.out_mode) k.push_back(static_cast<char>('0' + b));
  return k;
}

std::string kernel_name(const Spec &s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : cache_key(s)) h = (h ^ c) * 1099511628211ull;
  char name[96];
  std::snprintf(name, sizeof name, "rs_fft_%s_k%u_m%u_%016llx",
                s.inverse ? "inverse" : s.decode ? (s.present.empty() ? "decode" : "pdecode") : "encode", s.k, s.m,
                static_cast<unsigned long long>(h));
  return name;
}

std::string generate(const Spec &s, const std::string &name) { return gen_source(s, name, nullptr); }

uint32_t dyn_mask_words(const Spec &s) { return dyn_store_word(make_plan(s)) + 2; }

uint32_t decode_mask_offset(const Spec &s) { return (dyn_mask_words(s) + 3 + s.k + 15) & ~15u; }
uint32_t decode_block_words(const Spec &s) { return decode_mask_offset(s) + (s.m + s.k) * 128; }

namespace {
uint16_t gmul(uint16_t x, uint16_t y) { return x && y ? mul16(x, tables().log[y]) : 0; }
uint16_t tw_elem(uint64_t idx) {  // the element a butterfly multiplies by (0: XOR-only)
  const uint16_t l = sk(idx);
  return l == kModulus ? 0 : tables().exp[l];
}
}  // namespace

// The decode transform of root.zig:268-335 (W = ceilPow2(C + k) points) on a residual
// codeword that is zero outside positions [0, C): the IFFT's layers of distance >= C
// spread block 0 into every block as scalar multiples lambda_K of a = IFFT_C(block 0),
// the formal derivative adds lambda of the neighbouring blocks (its in-block part keeps
// the form lambda_K D_C(a)), and the FFT's layers of distance >= C combine blocks
// again. Tracking each block as alpha_K D_C(a) + beta_K a gives alpha_K = 0 for every
// data block, so block K's evaluations are beta_K FFT_{C, skew KC}(a).
bool decode_betas(uint32_t k, uint32_t m, std::vector<uint16_t> &beta) {
  const uint64_t C = ceil_pow2(m), W = ceil_pow2(C + k), nb = W / C;
  std::vector<uint16_t> lam(nb, 0), al(nb, 0), be(nb, 0);
  lam[0] = 1;
  for (uint64_t d = C; d < W; d *= 2)  // ifftPartial: y ^= x; x ^= t y (Generic.zig:171-192)
    for (uint64_t g = 0; g < W; g += 2 * d) {
      const uint16_t t = tw_elem(g + d - 1);
      for (uint64_t i = g; i < g + d; i += C) {
        const uint64_t x = i / C, y = (i + d) / C;
        lam[y] ^= lam[x];
        lam[x] ^= gmul(t, lam[y]);
      }
    }
  for (uint64_t K = 0; K < nb; K++) {  // root.zig:309-315: block K ^= raw block K | bit
    al[K] = lam[K];
    for (uint64_t b = 1; b < nb; b <<= 1)
      if (!(K & b)) be[K] ^= lam[K | b];
  }
  for (uint64_t d = W / 2; d >= C; d /= 2)  // fftPartial: x ^= t y; y ^= x (Generic.zig:149-169)
    for (uint64_t g = 0; g < W; g += 2 * d) {
      const uint16_t t = tw_elem(g + d - 1);
      for (uint64_t i = g; i < g + d; i += C) {
        const uint64_t x = i / C, y = (i + d) / C;
        al[x] ^= gmul(t, al[y]);
        be[x] ^= gmul(t, be[y]);
        al[y] ^= al[x];
        be[y] ^= be[x];
      }
    }
  beta = be;
  for (uint64_t K = 1; K < nb; K++)
    if (al[K]) return false;
  return true;
}

void uv_basis(uint32_t p[8]) {
  for (int i = 0; i < 8; i++) p[i] = basis().p[i];
}

void scalar_masks(uint16_t c, uint32_t *M) {
  std::memset(M, 0, 128 * sizeof(uint32_t));
  if (!c) return;
  const Tw t = twiddle(tables().log[c], false);
  for (int i = 0; i < 8; i++)
    for (int j = 0; j < 8; j++) {
      M[16 * i + j] = ((t.A[i] >> j & 1) ? 0x0F0F0F0Fu : 0u) | ((t.D[i] >> j & 1) ? 0xF0F0F0F0u : 0u);
      M[16 * i + 8 + j] = ((t.B[i] >> j & 1) ? 0x0F0F0F0Fu : 0u) | ((t.Cm[i] >> j & 1) ? 0xF0F0F0F0u : 0u);
    }
}

int decode_block(const Spec &s, const uint8_t *present, uint32_t *blk) {
  const uint32_t k = s.k, m = s.m, C = static_cast<uint32_t>(ceil_pow2(m));
  const uint32_t dwm = dyn_mask_words(s), mko = decode_mask_offset(s);
  std::memset(blk, 0, decode_block_words(s) * sizeof(uint32_t));
  std::vector<uint16_t> beta;
  if (!decode_betas(k, m, beta)) return RS_ERR_INVALID_ARGUMENT;
  uint32_t e = 0;
  for (uint32_t g = 0; g < k; g++) e += present[g] ? 0 : 1;
  std::vector<uint8_t> received(ceil_pow2(C + k), 0);
  uint32_t nr = 0;
  for (uint32_t p = 0; p < m && nr < e; p++)
    if (present[k + p]) {
      received[p] = 1;
      blk[dwm + 1 + p / 32] |= 1u << (p % 32);
      nr++;
    }
  if (nr < e) return RS_ERR_NOT_ENOUGH_SHARDS;
  uint32_t row = 0;
  for (uint32_t g = 0; g < k; g++) {
    received[C + g] = present[g] ? 1 : 0;
    blk[dwm + 3 + g] = present[g] ? 0xFFFFFFFFu : row++;
    if (!present[g]) {
      blk[g / 32] |= 1u << (g % 32);
      blk[dwm] |= 1u << ((C + g) / C);
    }
  }
  std::vector<uint16_t> er(kOrder);
  erasure_logs(received.data(), k, m, er.data());  // root.zig:277-289 (rows off R count as erased)
  const Tables &T = tables();
  for (uint32_t p = 0; p < m; p++)
    if (received[p]) scalar_masks(T.exp[er[p]], blk + mko + 128 * p);  // root.zig:292-295
  for (uint32_t g = 0; g < k; g++)
    if (!present[g])  // root.zig:321-326, with the block's beta
      scalar_masks(gmul(beta[(C + g) / C], T.exp[kModulus - er[C + g]]), blk + mko + 128 * (m + g));
  return RS_OK;
}

Stats stats(const Spec &s) {
  Stats st;
  (void)gen_source(s, "x", &st);
  return st;
}

const jit::Kernel *get(const Spec &s, bool async, std::string &err, bool &pending) {
  Spec copy = s;
  copy.prefetch = prefetch_of(s);
  copy.blocked = copy.blocked || walk_of();
  for (;;) {
    const std::string name = kernel_name(copy);
    const jit::Kernel *k =
        jit::get_source(cache_key(copy), name, [copy, name] { return generate(copy, name); }, async, err, pending);
    if (!k) return nullptr;
    int local = 0;
    if (hipFuncGetAttribute(&local, HIP_FUNC_ATTRIBUTE_LOCAL_SIZE_BYTES, k->fn) != hipSuccess) local = 0;
    // RS_AMD_FFT_ALLOW_SPILL=1: run a spilled build (tools/spill_repro.py, spill_root_cause.md)
    if (local && std::getenv("RS_AMD_FFT_ALLOW_SPILL")) return k;
    if (local == 0 || copy.prefetch == 0) {
      // a decode kernel of a long code (RS(1000,64): 16 blocks) may keep a few registers
      // in scratch even without prefetch; since the store-data hazard fix such builds are
      // bit-exact (spill_root_cause.md), and they beat every other reconstruct form there
      if (local && !copy.decode) {
        err = "FFT kernel spills registers even without prefetch";
        return nullptr;
      }
      return k;
    }
    copy.prefetch = copy.prefetch > 3 ? 3 : copy.prefetch > 2 ? 2 : 0;  // spilled: less prefetch (fewer live registers)
  }
}

bool compile_check(const Spec &s, std::string &err, double *ms, size_t *code_bytes) {
  const std::string name = kernel_name(s);
  const std::string src = generate(s, name);
  if (const char *dir = std::getenv("RS_AMD_JIT_DUMP")) {
    if (FILE *f = std::fopen((std::string(dir) + "/" + name + ".hip").c_str(), "w")) {
      std::fputs(src.c_str(), f);
      std::fclose(f);
    }
  }
  return jit::compile_source_check(src, err, ms, code_bytes);
}

hipError_t launch(const jit::Kernel &kn, const Spec &s, const uint8_t *data, uint64_t ds, const uint8_t *rec, uint64_t rs,
                  uint8_t *out, uint64_t os, uint64_t sb, uint64_t n_stripes, hipStream_t st, const uint32_t *dmask,
                  uint32_t dmask_words, bool shared_mask) {
  if (n_stripes == 0) return hipSuccess;
  if (!supports(s.k, s.m, sb, s.dyn || s.decode) || pieces(sb) != s.pieces ||
      (s.inverse && !supports_inverse(s.k, s.m, sb)))
    return hipErrorInvalidValue;
  if (s.dyn && (s.pieces != 1 || !dmask || dmask_words < (s.decode ? decode_block_words(s) : dyn_mask_words(s))))
    return hipErrorInvalidValue;
  if (s.decode && ((!s.dyn && s.present.empty()) || s.inverse || s.flags || !rec)) return hipErrorInvalidValue;
  const uint32_t C = static_cast<uint32_t>(ceil_pow2(s.m));
  static std::mutex mu;
  static std::map<int, int> cus;
  int dev = 0, n_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = cus.find(dev);
    if (it == cus.end()) {
      hipError_t e = hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
      if (e != hipSuccess) return e;
      cus[dev] = n_cu;
    } else {
      n_cu = it->second;
    }
  }
  uint32_t ups = s.pieces > 1 ? 1u : static_cast<uint32_t>(sb / kUnitBytes);
  uint64_t n_units = s.pieces > 1 ? (n_stripes + 1) / 2 : n_stripes * ups;
  uint64_t n_st = n_stripes;
  // one workgroup per CU (128 KiB of LDS for chunk 64), persistent over the units
  const uint32_t per_cu = C == 64 ? 1 : C == 32 ? 2 : 4;  // LDS 128 / 64 / 32 KiB per workgroup
  const uint64_t grid = std::min<uint64_t>(n_units, static_cast<uint64_t>(n_cu) * per_cu);
  uint32_t sb32 = static_cast<uint32_t>(sb);
  const unsigned char *d = data, *r = rec ? rec : data;
  unsigned char *o = out;
  const uint32_t *dm = dmask;
  uint32_t dmw = shared_mask ? 0u : dmask_words;  // the kernel's per-stripe mask stride
  unsigned long long *stamps = debug_of() & 64 ? stamp_buffer(dev) : nullptr;
  void *args[] = {&d, &ds, &r, &rs, &o, &os, &sb32, &ups, &n_units, &n_st, &dm, &dmw, &stamps};
  trace_launch(kn.name.c_str());
  return hipModuleLaunchKernel(kn.fn, static_cast<uint32_t>(grid), 1, 1, (C / 8) * 64, 1, 1, 0, st, args, nullptr);
}

int read_stamps(uint64_t *host, size_t n) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  unsigned long long *p = stamp_buffer(dev);
  if (!p || hipDeviceSynchronize() != hipSuccess) return -1;
  return hipMemcpy(host, p, std::min<size_t>(n, 8 * 64) * 8, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}

uint64_t selftest(const Spec &s, int trials) {
  Plan P = make_plan(s);
  std::mt19937_64 rng(12345);
  uint64_t bad = 0;
  const uint32_t C = P.C;
  auto apply = [&](std::vector<uint16_t> &v, const Layer &L) {
    for (const Bf &b : L.bf) {
      const Tw &t = P.get_tw(b.log_m);
      auto mulv = [&](uint16_t y) -> uint16_t {  // (u|v) coordinates through the kernel's blocks
        if (t.zero) return 0;
        uint16_t r = 0;
        for (int i = 0; i < 8; i++) {
          const uint8_t u = y & 0xFF, vv = y >> 8;
          const int lo = __builtin_popcount(t.A[i] & u) ^ __builtin_popcount(t.B[i] & vv);
          const int hi = __builtin_popcount(t.Cm[i] & u) ^ __builtin_popcount(t.D[i] & vv);
          r |= static_cast<uint16_t>((lo & 1) << i);
          r |= static_cast<uint16_t>((hi & 1) << (8 + i));
        }
        return r;
      };
      uint16_t &x = v[b.x], &y = v[b.y];
      if (L.inv) {
        y ^= x;
        x ^= mulv(y);
      } else {
        x ^= mulv(y);
        y ^= x;
      }
    }
  };
  for (int tr = 0; tr < trials; tr++) {
    std::vector<uint16_t> in(s.k);
    for (auto &x : in) x = static_cast<uint16_t>(rng());
    std::vector<uint16_t> ref(s.m), in_ref = in;
    for (uint32_t i = 0; i < s.k; i++)
      if (i < s.skip.size() && s.skip[i]) in_ref[i] = 0;
    scalar_encode(in_ref.data(), s.k, s.m, P.d1, (s.flags & RS_FLAG_QUIRK_D2) != 0, ref.data());
    std::vector<uint16_t> acc(C, 0);
    for (size_t j = 0; j < P.truncs.size(); j++) {
      std::vector<uint16_t> v(C, 0);
      for (uint32_t q = 0; q < C; q++) v[q] = P.valid[j][q] ? to_uv(in[j * C + q]) : 0;
      for (const Layer &L : P.ifft[j]) apply(v, L);
      for (uint32_t q = 0; q < C; q++) acc[q] ^= v[q];
    }
    for (const Layer &L : P.fft) apply(acc, L);
    if (s.inverse) {  // the kernel's output is data whose encode gives back `in`
      std::vector<uint16_t> data(s.k), par(s.m);
      for (uint32_t q = 0; q < s.k; q++) data[q] = to_uv(acc[q]);
      scalar_encode(data.data(), s.k, s.m, P.d1, (s.flags & RS_FLAG_QUIRK_D2) != 0, par.data());
      for (uint32_t q = 0; q < s.m; q++) bad += par[q] != in[q];
      continue;
    }
    for (uint32_t q = 0; q < s.m; q++) bad += to_uv(acc[q]) != ref[q];
  }
  return bad;
}

uint64_t decode_selftest(uint32_t k, uint32_t m, uint32_t e, int trials) {
  Spec s;
  s.k = k;
  s.m = m;
  s.dyn = s.decode = true;
  Plan P = make_plan(s);
  const uint32_t C = P.C, dwm = dyn_mask_words(s), mko = decode_mask_offset(s);
  std::mt19937_64 rng(777 + k * 131 + m * 7 + e);
  uint64_t bad = 0;
  auto apply = [&](std::vector<uint16_t> &v, const Layer &L) {  // the kernel's butterflies in (u|v) coordinates
    for (const Bf &b : L.bf) {
      const Tw &t = P.get_tw(b.log_m);
      auto mulv = [&](uint16_t y) -> uint16_t {
        if (t.zero) return 0;
        uint16_t r = 0;
        for (int i = 0; i < 8; i++) {
          const uint8_t u = y & 0xFF, vv = y >> 8;
          r |= static_cast<uint16_t>(((__builtin_popcount(t.A[i] & u) ^ __builtin_popcount(t.B[i] & vv)) & 1) << i);
          r |= static_cast<uint16_t>(((__builtin_popcount(t.Cm[i] & u) ^ __builtin_popcount(t.D[i] & vv)) & 1) << (8 + i));
        }
        return r;
      };
      uint16_t &x = v[b.x], &y = v[b.y];
      if (L.inv) {
        y ^= x;
        x ^= mulv(y);
      } else {
        x ^= mulv(y);
        y ^= x;
      }
    }
  };
  auto rmul = [](uint16_t x, const uint32_t *M) -> uint16_t {  // the kernel's rmul on one symbol
    const uint8_t u = x & 0xFF, v = x >> 8;
    uint16_t r = 0;
    for (int i = 0; i < 8; i++) {
      int lo = 0, hi = 0;
      for (int j = 0; j < 8; j++) {
        lo ^= ((u >> j & 1) && (M[16 * i + j] & 0x0F0F0F0Fu)) ^ ((v >> j & 1) && (M[16 * i + 8 + j] & 0x0F0F0F0Fu));
        hi ^= ((v >> j & 1) && (M[16 * i + j] & 0xF0F0F0F0u)) ^ ((u >> j & 1) && (M[16 * i + 8 + j] & 0xF0F0F0F0u));
      }
      r |= static_cast<uint16_t>(lo << i | hi << (8 + i));
    }
    return r;
  };
  std::vector<uint32_t> blk(decode_block_words(s));
  for (int tr = 0; tr < trials; tr++) {
    std::vector<uint16_t> data(k), par(m);
    for (auto &x : data) x = static_cast<uint16_t>(rng());
    scalar_encode(data.data(), k, m, false, false, par.data());
    std::vector<uint8_t> present(k + m, 1);
    std::vector<uint32_t> idx(k);
    for (uint32_t i = 0; i < k; i++) idx[i] = i;
    std::shuffle(idx.begin(), idx.end(), rng);
    for (uint32_t i = 0; i < e; i++) present[idx[i]] = 0;
    for (uint32_t p = 0; p < m - e; p++)  // drop some surplus recovery rows too
      if (rng() % 4 == 0) present[k + rng() % m] = 0;
    uint32_t have = 0;
    for (uint32_t p = 0; p < m; p++) have += present[k + p];
    if (have < e) continue;
    if (decode_block(s, present.data(), blk.data()) != RS_OK) return ~0ull;
    std::vector<uint16_t> d2 = data, enc(m);
    for (uint32_t g = 0; g < k; g++)
      if (!present[g]) d2[g] = 0;
    scalar_encode(d2.data(), k, m, false, false, enc.data());
    std::vector<uint16_t> a(C, 0);
    for (uint32_t p = 0; p < m; p++)
      if (blk[dwm + 1 + p / 32] >> (p % 32) & 1) a[p] = rmul(to_uv(par[p] ^ enc[p]), &blk[mko + 128 * p]);
    for (const Layer &L : ifft_layers(C, m, 0)) apply(a, L);
    for (uint32_t K = 1; K <= (k + C - 1) / C; K++) {
      if (!(blk[dwm] >> K & 1)) continue;
      const uint32_t tK = std::min<uint32_t>(C, k - (K - 1) * C);
      std::vector<uint16_t> y = a;
      for (const Layer &L : fft_layers(C, tK, static_cast<uint64_t>(K) * C)) apply(y, L);
      for (uint32_t q = 0; q < tK; q++) {
        const uint32_t g = (K - 1) * C + q;
        if (present[g]) continue;
        bad += to_uv(rmul(y[q], &blk[mko + 128 * (m + g)])) != data[g];
      }
    }
  }
  return bad;
}

}  // namespace fftnet
}  // namespace rs
