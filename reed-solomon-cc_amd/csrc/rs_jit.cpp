// rs_jit.cpp — generator, hipRTC compiler and launcher of the bit-sliced
// network kernels (rs_jit.hpp).
#include "rs_jit.hpp"

#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <sstream>
#include <thread>

#include "rs_internal.hpp"

namespace rs {
namespace jit {
namespace {

// Device-side helpers shared by every generated kernel.
//  * ld / st: a wave covers 4 KiB of a shard = two 2 KiB regions of the
//    contiguous lane layout of rs_device.hpp (lanes 0-31 read the lo halves,
//    32-63 the hi halves of 16 consecutive 64-B chunks, 1 KiB per instruction),
//    then one v_permlane32_swap per dword pairs every lane's lo and hi dwords.
//    Lane result: lo[8] (lo bytes of 32 symbols) and hi[8] (their hi bytes).
//  * tr8: in-place 8x8 bit transpose of every byte lane of x[0..8):
//    afterwards bit b of byte q of x[j] = bit j of byte q of the input x[b],
//    i.e. x[j] is bit-plane j of the 32 symbols (symbol of byte q of dword b at
//    bit 8q+b, the same position in every plane). Three delta-swap stages of
//    one shift + one v_bitop3 mux per word; an involution, so it also undoes
//    itself on the way out.
const char *kPrelude = R"HIP(
typedef unsigned int u32;
typedef unsigned long long u64;
typedef u32 v4 __attribute__((ext_vector_type(4)));
#define X3(a, b, c) __builtin_amdgcn_bitop3_b32((a), (b), (c), 0x96)
#define MUX(a, b, m) __builtin_amdgcn_bitop3_b32((a), (b), (m), 0xE4)
#define TRS(j, d, m)                 \
  {                                  \
    const u32 a = x[j], b = x[j + d]; \
    x[j] = MUX(a, b << d, m);        \
    x[j + d] = MUX(a >> d, b, m);    \
  }
// the transpose masks in VGPRs when RS_VMASK (a v_bitop3 with an SGPR source issues at ~2/3
// rate with two or more waves per SIMD, profiles/r04/valu_probe2.log; VOP3 takes no literal)
#if RS_VMASK
#define KMASK(c) ({ u32 m_ = (c); asm("" : "+v"(m_)); m_; })
#else
#define KMASK(c) (c)
#endif
__device__ __forceinline__ void tr8(u32 *x) {
  const u32 f = KMASK(0x0F0F0F0Fu), t = KMASK(0x33333333u), s = KMASK(0x55555555u);
  TRS(0, 4, f) TRS(1, 4, f) TRS(2, 4, f) TRS(3, 4, f)
  TRS(0, 2, t) TRS(1, 2, t) TRS(4, 2, t) TRS(5, 2, t)
  TRS(0, 1, s) TRS(2, 1, s) TRS(4, 1, s) TRS(6, 1, s)
}
#if RS_NT & 1
#define LDV(p) __builtin_nontemporal_load((const v4 *)(p))
#else
#define LDV(p) (*(const v4 *)(p))
#endif
#if RS_NT & 2
#define STV(v, p) __builtin_nontemporal_store((v), (v4 *)(p))
#else
#define STV(v, p) (*(v4 *)(p) = (v))
#endif
struct Raw { v4 a0, a1, b0, b1; };
__device__ __forceinline__ Raw ld(const unsigned char *p) {
  Raw r;
  r.a0 = LDV(p);
  r.a1 = LDV(p + 1024);
  r.b0 = LDV(p + 2048);
  r.b1 = LDV(p + 3072);
  return r;
}
// p ^ q before the plane transform (a bit permutation, so it commutes with XOR)
__device__ __forceinline__ Raw ldx(const unsigned char *p, const unsigned char *q) {
  Raw r = ld(p);
  const Raw t = ld(q);
  r.a0 ^= t.a0;
  r.a1 ^= t.a1;
  r.b0 ^= t.b0;
  r.b1 ^= t.b1;
  return r;
}
__device__ __forceinline__ void planes(const Raw &r, u32 *P) {
#pragma unroll
  for (int v = 0; v < 4; v++) {
    const auto s = __builtin_amdgcn_permlane32_swap(r.a0[v], r.a1[v], false, false);
    const auto t = __builtin_amdgcn_permlane32_swap(r.b0[v], r.b1[v], false, false);
    P[v] = s[0];
    P[8 + v] = s[1];
    P[4 + v] = t[0];
    P[12 + v] = t[1];
  }
  tr8(P);
  tr8(P + 8);
}
__device__ __forceinline__ void st(unsigned char *p, u32 *P) {
  tr8(P);
  tr8(P + 8);
  v4 a0, a1, b0, b1;
#pragma unroll
  for (int v = 0; v < 4; v++) {
    const auto s = __builtin_amdgcn_permlane32_swap(P[v], P[8 + v], false, false);
    const auto t = __builtin_amdgcn_permlane32_swap(P[4 + v], P[12 + v], false, false);
    a0[v] = s[0];
    a1[v] = s[1];
    b0[v] = t[0];
    b1[v] = t[1];
  }
  STV(a0, p);
  STV(a1, p + 1024);
  STV(b0, p + 2048);
  STV(b1, p + 3072);
}
)HIP";

// Small shards (NetSpec::pieces > 1): the four 1 KiB pieces of a wave unit sit in
// different stripes, so loads and stores take one base pointer per piece. A piece
// of a stripe past the batch is clamped to the last stripe, which lies in the same
// unit: it reads the same bytes as that stripe's piece at the same offset, so its
// store rewrites identical values there (branch-free: guarding the stores with
// branches made the compiler keep every input's temporaries live, 512 VGPRs + spills).
const char *kPreludeSmall = R"HIP(
__device__ __forceinline__ Raw ld4(const unsigned char *const *p, u32 x) {
  Raw r;
  r.a0 = LDV(p[0] + x);
  r.a1 = LDV(p[1] + x);
  r.b0 = LDV(p[2] + x);
  r.b1 = LDV(p[3] + x);
  return r;
}
__device__ __forceinline__ Raw ldx4(const unsigned char *const *p, const unsigned char *const *q, u32 x) {
  Raw r = ld4(p, x);
  const Raw t = ld4(q, x);
  r.a0 ^= t.a0;
  r.a1 ^= t.a1;
  r.b0 ^= t.b0;
  r.b1 ^= t.b1;
  return r;
}
__device__ __forceinline__ void st4(unsigned char *const *p, u32 x, u32 *P) {
  tr8(P);
  tr8(P + 8);
  v4 a0, a1, b0, b1;
#pragma unroll
  for (int v = 0; v < 4; v++) {
    const auto s = __builtin_amdgcn_permlane32_swap(P[v], P[8 + v], false, false);
    const auto t = __builtin_amdgcn_permlane32_swap(P[4 + v], P[12 + v], false, false);
    a0[v] = s[0];
    a1[v] = s[1];
    b0[v] = t[0];
    b1[v] = t[1];
  }
  STV(a0, p[0] + x);
  STV(a1, p[1] + x);
  STV(b0, p[2] + x);
  STV(b1, p[3] + x);
}
)HIP";

// XOR network of one input's 16 planes into up to 64 accumulator planes.
// Four-Russians style: planes in groups of 4; per group every distinct nonzero
// sub-row a row needs is built once (1 op each from the singles), then every
// accumulator takes one XOR3 per pair of groups.
void emit_input(std::ostringstream &o, const std::vector<uint16_t> &rows, std::vector<bool> &init, int t) {
  const size_t n = rows.size();
  for (int pair = 0; pair < 2; pair++) {
    std::string name[2][16];
    for (int h = 0; h < 2; h++) {
      const int g = 2 * pair + h;
      bool need[16] = {};
      for (size_t r = 0; r < n; r++) need[(rows[r] >> (4 * g)) & 15] = true;
      auto single = [&](int i) { return "P[" + std::to_string(4 * g + i) + "]"; };
      for (int i = 0; i < 4; i++) name[h][1 << i] = single(i);
      // pairs first (so that 4-element combos can reuse one)
      for (int msk = 1; msk < 16; msk++) {
        const int pc = __builtin_popcount(msk);
        if (!need[msk] || pc != 2) continue;
        int b[2], nb = 0;
        for (int i = 0; i < 4; i++)
          if (msk >> i & 1) b[nb++] = i;
        name[h][msk] = "c" + std::to_string(t) + "_" + std::to_string(g) + "_" + std::to_string(msk);
        o << "  const u32 " << name[h][msk] << " = " << single(b[0]) << " ^ " << single(b[1]) << ";\n";
      }
      for (int msk = 1; msk < 16; msk++) {
        const int pc = __builtin_popcount(msk);
        if (!need[msk] || pc < 3) continue;
        name[h][msk] = "c" + std::to_string(t) + "_" + std::to_string(g) + "_" + std::to_string(msk);
        o << "  const u32 " << name[h][msk] << " = ";
        if (pc == 3) {
          int b[3], nb = 0;
          for (int i = 0; i < 4; i++)
            if (msk >> i & 1) b[nb++] = i;
          o << "X3(" << single(b[0]) << ", " << single(b[1]) << ", " << single(b[2]) << ");\n";
        } else {
          static const int pairs[6][2] = {{3, 12}, {12, 3}, {5, 10}, {10, 5}, {6, 9}, {9, 6}};
          bool done = false;
          for (auto &pp : pairs)
            if (!name[h][pp[0]].empty() && name[h][pp[0]][0] == 'c') {
              const int r0 = __builtin_ctz(pp[1]), r1 = 31 - __builtin_clz(pp[1]);
              o << "X3(" << name[h][pp[0]] << ", " << single(r0) << ", " << single(r1) << ");\n";
              done = true;
              break;
            }
          if (!done) o << "X3(" << single(0) << ", " << single(1) << ", " << single(2) << ") ^ " << single(3) << ";\n";
        }
      }
    }
    for (size_t r = 0; r < n; r++) {
      std::string terms[2];
      int nt = 0;
      for (int h = 0; h < 2; h++) {
        const int sub = (rows[r] >> (4 * (2 * pair + h))) & 15;
        if (sub) terms[nt++] = name[h][sub];
      }
      if (!nt) continue;
      const std::string acc = "a" + std::to_string(r);
      if (!init[r]) {
        o << "  " << acc << " = " << terms[0];
        if (nt == 2) o << " ^ " << terms[1];
        o << ";\n";
        init[r] = true;
      } else if (nt == 1) {
        o << "  " << acc << " ^= " << terms[0] << ";\n";
      } else {
        o << "  " << acc << " = X3(" << acc << ", " << terms[0] << ", " << terms[1] << ");\n";
      }
    }
  }
}

// Code shape. Constants measured in rounds 1-2 (profiles/r01/sweep_net_*.jsonl): no input
// prefetch (the compiler hoists the loads anyway), no occupancy hint, non-temporal loads
// and stores for one-tile maps (stores only for several tiles: their inputs are re-read
// through L2), one 4 KiB unit per wave, sched_barriers between inputs above 16 input
// blocks (bounds the scheduling regions: compile time stays ~linear in size). The knobs
// the tests use to reach the other forms (read at generation time, part of the cache key):
//   RS_AMD_NET_TILE      outputs per workgroup, 4 (64 accumulator planes) or 8 (default:
//                        half the input re-reads and plane transforms of multi-tile maps;
//                        RS(32,8) encode 2.39 -> 1.91 ms, the 55 x 55 syndrome map
//                        13.9 -> 12.3 ms reconstruct, profiles/r01/sweep_net_tile8.jsonl)
//   RS_AMD_NET_SHARED    0: the classic form instead of the shared-input form
//   RS_AMD_NET_BALANCE   0: one wave per 8-output tile in the shared form
struct Tuning {
  int prefetch = 0, waves = 0, nt = 3, barrier = -1, units = 1, tile = 8, shared = -1, balance = 1, vmask = 1;
};

int env_int(const char *name, int def) {
  const char *e = std::getenv(name);
  return e && *e ? std::atoi(e) : def;
}

Tuning tuning() {
  Tuning t;
  t.tile = env_int("RS_AMD_NET_TILE", t.tile) >= 8 ? 8 : 4;
  t.shared = env_int("RS_AMD_NET_SHARED", t.shared);
  t.balance = env_int("RS_AMD_NET_BALANCE", t.balance) != 0;
  t.vmask = env_int("RS_AMD_NET_VMASK", t.vmask) != 0;
  return t;
}

std::string tuning_key(const Tuning &t) {
  return "t" + std::to_string(t.tile) + "s" + std::to_string(t.shared) + (t.balance ? "" : "nb") + (t.vmask ? "" : "nv");
}

// Shared-input form (generate_shared): one workgroup of n_tiles waves per 4 KiB unit,
// the inputs' plane transforms done once and shared through LDS. RS_AMD_NET_SHARED:
// 0 off, else (default) on for 2..8 output tiles of whole 4 KiB units. Measured
// (profiles/r02/sweep_shared_net.jsonl): the RS(200,55) 55 x 55 syndrome map 8.43 ->
// 6.84 ms reconstruct, RS(16,16) 1 MiB encode 4.16 -> 3.44 ms, RS(64,64) losing 40
// 3.92 -> 3.26 ms, RS(200,55) losing 20 6.35 -> 5.21 ms.
bool shared_on(const Tuning &t, const NetSpec &spec) {
  const uint32_t n_tiles = (spec.n_out + t.tile - 1) / t.tile;
  return spec.pieces == 1 && n_tiles >= 2 && n_tiles <= 8 && t.shared != 0;
}

// Waves per workgroup of the shared form. Its ~200-VGPR waves fit two per SIMD, and a
// workgroup's waves advance together (one barrier per batch), so a workgroup of 3 or
// 5..7 waves leaves SIMDs holding one wave fewer than the others for the whole kernel
// (7 waves: 2,2,2,1). RS_AMD_NET_BALANCE (default on) rounds the wave count up to 4 or
// 8 and spreads the outputs evenly (55 outputs: 8 tiles of 7/6 instead of 7 of 8/7).
uint32_t shared_tiles(const Tuning &t, const NetSpec &spec) {
  const uint32_t n_tiles = (spec.n_out + t.tile - 1) / t.tile;
  if (!t.balance) return n_tiles;
  return n_tiles == 3 ? std::min(4u, spec.n_out) : n_tiles >= 5 ? std::min(8u, spec.n_out) : n_tiles;
}

uint32_t kernel_tiles(const Tuning &t, const NetSpec &spec) {
  return shared_on(t, spec) ? shared_tiles(t, spec) : (spec.n_out + t.tile - 1) / t.tile;
}

}  // namespace

bool net_vmask() { return env_int("RS_AMD_NET_VMASK", 1) != 0; }
std::string net_prelude() { return std::string("#define RS_VMASK ") + (net_vmask() ? "1\n" : "0\n") + kPrelude; }
void emit_network_input(std::ostringstream &o, const std::vector<uint16_t> &rows, std::vector<bool> &init, int t) {
  emit_input(o, rows, init, t);
}

uint64_t max_blocks() { return kMaxBlocks; }

bool supports(uint32_t n_in, uint32_t n_out, uint64_t shard_bytes) {
  const uint64_t blocks = static_cast<uint64_t>(n_in) * ((n_out + kTileOut - 1) / kTileOut);
  return n_in > 0 && n_out > 0 && n_out <= kMaxOut && blocks <= max_blocks() && shard_ok(shard_bytes);
}

// RS_AMD_NET_SMALL=0 keeps 1 / 2 KiB shards on the table kernels
bool shard_ok(uint64_t shard_bytes) {
  if (shard_bytes == 1024 || shard_bytes == 2048) return env_int("RS_AMD_NET_SMALL", 1) != 0;
  return shard_bytes > 0 && shard_bytes % kUnitBytes == 0 && shard_bytes < (1ull << 32);
}

uint32_t net_pieces(uint64_t shard_bytes) {
  return shard_bytes && shard_bytes < kUnitBytes ? static_cast<uint32_t>(kUnitBytes / shard_bytes) : 1u;
}

namespace {
std::string generate_with(const NetSpec &spec, const std::string &name, const Tuning &tu);
}

std::string generate(const NetSpec &spec, const std::string &name) { return generate_with(spec, name, tuning()); }

namespace {
// Shared-input network: a workgroup of T = n_tiles waves covers one 4 KiB unit of a
// stripe; wave w owns output tile w (its accumulators and its network code). Inputs go
// in batches of T: wave w loads input bT + w (prefetched one batch ahead), transforms it
// to planes and writes them to LDS (double-buffered, one barrier per batch), then every
// wave runs its tile's network over the batch's T inputs read back from LDS. Every input
// is read from HBM and transposed once instead of once per tile.
std::string generate_shared(const NetSpec &spec, const std::string &name, const Tuning &tu) {
  const uint32_t n_in = spec.n_in, n_out = spec.n_out;
  // one input staged per wave between barriers (two staged inputs per wave measured slower:
  // 8.25 vs 6.84 ms on the c4 55 x 55 map, 240 VGPRs)
  const uint32_t T = shared_tiles(tu, spec);
  // tile w owns outputs [w * n_out / T, (w + 1) * n_out / T)
  auto tile_first = [&](uint32_t w) { return static_cast<uint32_t>(static_cast<uint64_t>(w) * n_out / T); };
  const uint32_t mult = 1;
  const uint32_t BW = T * mult, nb = (n_in + BW - 1) / BW;
  std::ostringstream o;
  o << "#define RS_NT " << tu.nt << "\n#define RS_VMASK " << tu.vmask << "\n" << kPrelude;
  o << "extern \"C\" __global__ __launch_bounds__(" << 64 * T << ") ";
  if (tu.waves) o << "__attribute__((amdgpu_waves_per_eu(" << tu.waves << ", 8))) ";
  o << "void " << name
    << "(const unsigned char *__restrict__ b0, u64 s0, const unsigned char *__restrict__ b1, u64 s1,\n"
       "    unsigned char *__restrict__ out, u64 so, u64 sb, u64 stripe0,\n"
       "    const unsigned char *__restrict__ b2, u64 s2, u64 nst) {\n"
    << "  __shared__ v4 xs[" << 2 * BW * 4 * 64 << "];\n"
       "  const u32 lane = threadIdx.x & 63u, ll = lane & 31u;\n"
       "  const u32 w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);\n"
       "  const u64 s = stripe0 + blockIdx.y;\n"
       "  const unsigned char *B0 = b0 + s * s0, *B1 = b1 + s * s1, *B2 = b2 + s * s2;\n"
       "  unsigned char *O = out + s * so;\n"
       "  const u32 off = blockIdx.x * 4096u + (ll >> 1) * 64u + (lane >= 32u ? 32u : 0u) + (ll & 1u) * 16u;\n";
  auto load_expr = [&](uint32_t t) {
    const int32_t src = spec.src[t];
    const uint32_t idx = static_cast<uint32_t>(src & kSrcIndexMask);
    std::ostringstream e;
    if (src & kSrcXorScratch)
      e << "ldx(B1 + " << idx << "ull * sb + off, B2 + " << idx << "ull * sb + off)";
    else
      e << "ld(" << ((src & kSrcRecovery) ? "B1" : "B0") << " + " << idx << "ull * sb + off)";
    return e.str();
  };

  // one complete path per tile (wave w = tile w): its staging of input bT + w, the
  // barrier, its network over the batch, for every batch. Disjoint paths keep the
  // register allocation per tile (one shared path with a branch per batch and tile
  // merged the tiles' live ranges: 372 VGPRs and spills for RS(32,32)); every path
  // passes the same number of barriers.
  for (uint32_t tile = 0; tile < T; tile++) {
    const uint32_t j0 = tile_first(tile), nj = tile_first(tile + 1) - j0;
    o << "  " << (tile ? "else if" : "if") << " (w == " << tile << "u) {\n  u32 ";
    for (size_t r = 0; r < 16 * nj; r++) o << "a" << r << (r + 1 < 16 * nj ? ", " : ";\n");
    std::vector<bool> init(16 * nj, false);
    for (uint32_t q = 0; q < mult; q++)  // inputs tile + qT of batch 0
      if (tile + q * T < n_in) o << "  Raw R" << q << " = " << load_expr(tile + q * T) << ";\n";
    for (uint32_t bt = 0; bt < nb; bt++) {
      const uint32_t buf = bt & 1, cnt = std::min(BW, n_in - bt * BW);
      o << "  // ---- batch " << bt << ": inputs " << bt * BW << ".." << bt * BW + cnt - 1 << "\n";
      for (uint32_t q = 0; q < mult; q++) {
        const uint32_t slot = tile + q * T;
        if (slot >= cnt) continue;
        o << "  {\n  u32 P[16];\n  planes(R" << q << ", P);\n";
        for (int qq = 0; qq < 4; qq++)
          o << "  xs[" << (buf * BW + slot) * 256 + qq * 64 << "u + lane] = (v4){P[" << 4 * qq << "], P[" << 4 * qq + 1
            << "], P[" << 4 * qq + 2 << "], P[" << 4 * qq + 3 << "]};\n";
        o << "  }\n";
        if ((bt + 1) * BW + slot < n_in) o << "  R" << q << " = " << load_expr((bt + 1) * BW + slot) << ";\n";
      }
      o << "  __builtin_amdgcn_fence(__ATOMIC_RELEASE, \"workgroup\", \"local\");\n"
           "  __builtin_amdgcn_s_barrier();\n"
           "  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"workgroup\", \"local\");\n";
      for (uint32_t i = 0; i < cnt; i++) {
        const uint32_t t = bt * BW + i;
        o << "  {\n  u32 P[16];\n";
        for (int q = 0; q < 4; q++)
          o << "  { const v4 x = xs[" << (buf * BW + i) * 256 + q * 64 << "u + lane]; P[" << 4 * q << "] = x[0]; P["
            << 4 * q + 1 << "] = x[1]; P[" << 4 * q + 2 << "] = x[2]; P[" << 4 * q + 3 << "] = x[3]; }\n";
        std::vector<uint16_t> rows(16 * nj, 0);
        for (uint32_t jj = 0; jj < nj; jj++)
          for (int bb = 0; bb < 16; bb++) {
            const uint16_t img = spec.images[(static_cast<size_t>(t) * n_out + j0 + jj) * 16 + bb];
            for (int c = 0; c < 16; c++)
              if (img >> c & 1) rows[jj * 16 + c] |= static_cast<uint16_t>(1u << bb);
          }
        emit_input(o, rows, init, static_cast<int>(t));
        o << "  }\n  __builtin_amdgcn_sched_barrier(0);\n";
      }
    }
    for (size_t r = 0; r < 16 * nj; r++)
      if (!init[r]) o << "  a" << r << " = 0u;\n";
    for (uint32_t jj = 0; jj < nj; jj++) {
      o << "  { u32 Q[16] = {";
      for (int c = 0; c < 16; c++) o << "a" << jj * 16 + c << (c < 15 ? ", " : "};\n");
      o << "    st(O + " << (j0 + jj) << "ull * sb + off, Q); }\n";
    }
    o << "  }\n";
  }
  o << "}\n";
  return o.str();
}

// the knobs are captured when a compile is requested (a background job must not see
// the environment of a later moment: the cache key already names these values)
std::string generate_with(const NetSpec &spec, const std::string &name, const Tuning &tu) {
  if (shared_on(tu, spec)) return generate_shared(spec, name, tu);
  const uint32_t n_in = spec.n_in, n_out = spec.n_out;
  const uint32_t tw = static_cast<uint32_t>(tu.tile);  // outputs per workgroup
  const uint32_t n_tiles = (n_out + tw - 1) / tw;
  std::ostringstream o;
  // several output tiles re-read every input through L2: non-temporal loads (which
  // evict early) cost 10-15 % there, so by default they are kept for 1-tile maps only
  const int nt = n_tiles == 1 ? tu.nt : (tu.nt & 2);
  const uint32_t P = spec.pieces;  // stripes per wave unit (1, or 2 / 4 for 2 / 1 KiB shards)
  o << "#define RS_NT " << nt << "\n#define RS_VMASK " << tu.vmask << "\n" << kPrelude;
  if (P > 1) o << kPreludeSmall;
  o << "extern \"C\" __global__ __launch_bounds__(256) ";
  if (tu.waves) o << "__attribute__((amdgpu_waves_per_eu(" << tu.waves << ", 8))) ";
  o << "void " << name
    << "(const unsigned char *__restrict__ b0, u64 s0, const unsigned char *__restrict__ b1, u64 s1,\n"
       "    unsigned char *__restrict__ out, u64 so, u64 sb, u64 stripe0,\n"
       "    const unsigned char *__restrict__ b2, u64 s2, u64 nst) {\n"
       "  const u32 lane = threadIdx.x & 63;\n"
    // XCD-aware: workgroups are dealt round-robin over the 8 XCDs (each with its own
    // L2), so the n_tiles workgroups of one unit group sit 8 apart in blockIdx.x (same
    // XCD, dispatched back to back): their input reads after the first hit that L2
    << "  const u32 bx = blockIdx.x, tile = (bx / 8u) % " << n_tiles << "u;\n"
    << "  const u64 ugroup = (u64)(bx / 8u / " << n_tiles << "u) * 8u + (bx % 8u);\n"
    << "  const u64 ubase = (ugroup * 4 + (threadIdx.x >> 6)) * " << tu.units << "u;\n"
       "  const u32 ll = lane & 31;\n";
  if (P == 1) {
    o << "  const u64 s = stripe0 + blockIdx.y;\n"
         "  const unsigned char *B0 = b0 + s * s0;\n"
         "  const unsigned char *B1 = b1 + s * s1;\n"
         "  const unsigned char *B2 = b2 + s * s2;\n"
         "  unsigned char *O = out + s * so;\n"
      << "#pragma unroll 1\n"
      << "  for (u32 it = 0; it < " << tu.units << "u; it++) {\n"
         "  const u64 unit = ubase + it;\n"
         "  if (unit * 4096 >= sb) break;\n"
         "  const u32 off = (u32)unit * 4096u + (ll >> 1) * 64u + (lane >= 32 ? 32u : 0u) + (ll & 1) * 16u;\n";
  } else {
    // unit u covers stripes [u*P, u*P + P) of the launch (blockIdx.y == 0); piece i
    // (1 KiB) lies in stripe u*P + i/(4/P) at shard offset (i % (4/P)) KiB
    const uint32_t per = 4 / P;  // pieces per stripe
    o << "#pragma unroll 1\n"
      << "  for (u32 it = 0; it < " << tu.units << "u; it++) {\n"
         // wave-uniform (readfirstlane): the piece pointers stay in SGPRs, loads use saddr + voffset
         "  const u64 unit = (ugroup * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) * "
      << tu.units << "u + it;\n"
      << "  const u64 sf = stripe0 + unit * " << P << "u;\n"
         "  if (sf >= nst) break;\n"
         "  const u32 off = (ll >> 1) * 64u + (lane >= 32 ? 32u : 0u) + (ll & 1) * 16u;\n"
         "  const unsigned char *B0[4], *B1[4], *B2[4];\n"
         "  unsigned char *O[4];\n";
    for (uint32_t i = 0; i < 4; i++) {
      o << "  { const u64 q = sf + " << i / per << "u;\n"
        << "    const u64 c = q < nst ? q : nst - 1, po = " << (i % per) * 1024 << "u;\n"
        << "    B0[" << i << "] = b0 + c * s0 + po; B1[" << i << "] = b1 + c * s1 + po;\n"
        << "    B2[" << i << "] = b2 + c * s2 + po; O[" << i << "] = out + c * so + po; }\n";
    }
  }
  auto load_expr = [&](uint32_t t) {  // ld(shard) or ldx(shard, scratch) for a syndrome input
    const int32_t src = spec.src[t];
    const uint32_t idx = static_cast<uint32_t>(src & kSrcIndexMask);
    std::ostringstream e;
    if (P > 1 && (src & kSrcXorScratch))
      e << "ldx4(B1, B2, " << idx << "u * (u32)sb + off)";
    else if (P > 1)
      e << "ld4(" << ((src & kSrcRecovery) ? "B1" : "B0") << ", " << idx << "u * (u32)sb + off)";
    else if (src & kSrcXorScratch)
      e << "ldx(B1 + " << idx << "ull * sb + off, B2 + " << idx << "ull * sb + off)";
    else
      e << "ld(" << ((src & kSrcRecovery) ? "B1" : "B0") << " + " << idx << "ull * sb + off)";
    return e.str();
  };
  for (uint32_t tile = 0; tile < n_tiles; tile++) {
    const uint32_t j0 = tile * tw, nj = std::min(tw, n_out - j0);
    const size_t n_acc = 16 * nj;
    o << "  " << (tile ? "else if" : "if") << " (tile == " << tile << "u) {\n";
    o << "  u32 ";
    for (size_t r = 0; r < n_acc; r++) o << "a" << r << (r + 1 < n_acc ? ", " : ";\n");
    std::vector<bool> init(n_acc, false);
    // input t + prefetch is loaded just before input t is transformed
    const uint32_t ahead = static_cast<uint32_t>(tu.prefetch);
    for (uint32_t t = 0; t < n_in; t++) {
      for (uint32_t u = t ? t + ahead : 0; u <= t + ahead && u < n_in; u++)
        o << "  const Raw R" << u << " = " << load_expr(u) << ";\n";
      o << "  {\n";
      o << "  u32 P[16];\n  planes(R" << t << ", P);\n";
      std::vector<uint16_t> rows(n_acc, 0);
      for (uint32_t jj = 0; jj < nj; jj++)
        for (int b = 0; b < 16; b++) {
          const uint16_t img = spec.images[(static_cast<size_t>(t) * n_out + j0 + jj) * 16 + b];
          for (int c = 0; c < 16; c++)
            if (img >> c & 1) rows[jj * 16 + c] |= static_cast<uint16_t>(1u << b);
        }
      emit_input(o, rows, init, static_cast<int>(t));
      o << "  }\n";
      // bound the scheduler's regions (compile time grows superlinearly with them)
      if (tu.barrier > 0 || (tu.barrier < 0 && n_in * n_tiles > 16)) o << "  __builtin_amdgcn_sched_barrier(0);\n";
    }
    for (size_t r = 0; r < n_acc; r++)
      if (!init[r]) o << "  a" << r << " = 0u;\n";
    for (uint32_t jj = 0; jj < nj; jj++) {
      o << "  { u32 Q[16] = {";
      for (int c = 0; c < 16; c++) o << "a" << jj * 16 + c << (c < 15 ? ", " : "};\n");
      if (P > 1)
        o << "    st4(O, " << (j0 + jj) << "u * (u32)sb + off, Q); }\n";
      else
        o << "    st(O + " << (j0 + jj) << "ull * sb + off, Q); }\n";
    }
    o << "  }\n";
  }
  o << "  }\n}\n";  // unit loop, kernel
  return o.str();
}
}  // namespace

// ------------------------------------------------------------- compile + cache
namespace {

std::mutex g_mu;
std::condition_variable g_cv;                              // signalled when a background compile ends
std::map<std::string, std::unique_ptr<Kernel>> g_cache;  // key: device + spec bytes
std::map<std::string, std::string> g_failed;              // key -> compile error (background compiles)
std::set<std::string> g_pending;                          // keys compiling in the background

std::string spec_key(const NetSpec &s, int dev, const Tuning &tu) {
  std::string k = std::to_string(dev) + ":" + s.role + ":" + tuning_key(tu) + ":" + std::to_string(s.n_in) + ":" +
                  std::to_string(s.n_out) + ":" + (s.pieces > 1 ? "p" + std::to_string(s.pieces) + ":" : "");
  k.append(reinterpret_cast<const char *>(s.src.data()), s.src.size() * sizeof(int32_t));
  k.append(reinterpret_cast<const char *>(s.images.data()), s.images.size() * sizeof(uint16_t));
  return k;
}

uint64_t fnv1a(const std::string &s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}

std::string kernel_name(const NetSpec &spec, const std::string &key) {
  char name[96];
  std::snprintf(name, sizeof name, "rs_net_%s_i%u_o%u_%016llx", spec.role.c_str(), spec.n_in, spec.n_out,
                static_cast<unsigned long long>(fnv1a(key)));
  return name;
}

// On-disk code-object cache: $RS_AMD_CACHE_DIR (empty = off), else
// $XDG_CACHE_HOME/rs_amd or ~/.cache/rs_amd. An entry is named by two 64-bit hashes
// of (hipRTC version, options, source) and its source length, so a process restart,
// another rank or another thread finds the code object instead of recompiling.
std::string cache_dir() {
  if (const char *d = std::getenv("RS_AMD_CACHE_DIR")) return d;
  if (const char *x = std::getenv("XDG_CACHE_HOME"))
    if (*x) return std::string(x) + "/rs_amd";
  if (const char *h = std::getenv("HOME"))
    if (*h) return std::string(h) + "/.cache/rs_amd";
  return "";
}

std::atomic<uint64_t> g_compiles{0}, g_disk_hits{0};

std::string cache_path(const std::string &dir, const std::string &src, const char *const *opts, int n_opts) {
  int major = 0, minor = 0;
  hiprtcVersion(&major, &minor);
  std::string id = "hiprtc " + std::to_string(major) + "." + std::to_string(minor) + "\n";
  for (int i = 0; i < n_opts; i++) id += std::string(opts[i]) + "\n";
  id += src;
  uint64_t h1 = 1469598103934665603ull, h2 = 0x9E3779B97F4A7C15ull;
  for (unsigned char c : id) {
    h1 = (h1 ^ c) * 1099511628211ull;
    h2 = (h2 ^ c) * 0x100000001B3ull + 0x2545F4914F6CDD1Dull;
  }
  char name[96];
  std::snprintf(name, sizeof name, "/%016llx%016llx-%zu.co", static_cast<unsigned long long>(h1),
                static_cast<unsigned long long>(h2), id.size());
  return dir + name;
}

// A code object is an ELF (or a clang offload bundle); anything else (a truncated or
// foreign file) is not loaded.
bool code_object_ok(const std::vector<char> &code) {
  static const char kElf[4] = {0x7F, 'E', 'L', 'F'};
  static const char kBundle[] = "__CLANG_OFFLOAD_BUNDLE__";
  if (code.size() >= 64 && std::memcmp(code.data(), kElf, 4) == 0) return true;
  return code.size() >= sizeof kBundle && std::memcmp(code.data(), kBundle, sizeof kBundle - 1) == 0;
}

bool cache_read(const std::string &path, std::vector<char> &code) {
  FILE *f = std::fopen(path.c_str(), "rb");
  if (!f) return false;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  bool ok = n > 0;
  if (ok) {
    code.resize(static_cast<size_t>(n));
    ok = std::fread(code.data(), 1, code.size(), f) == code.size();
  }
  std::fclose(f);
  if (ok && !code_object_ok(code)) {  // a bad entry is dropped and recompiled
    std::remove(path.c_str());
    ok = false;
  }
  return ok;
}

void cache_write(const std::string &dir, const std::string &path, const std::vector<char> &code) {
  std::string cur;  // mkdir -p
  for (size_t i = 0; i <= dir.size(); i++) {
    if (i == dir.size() || dir[i] == '/') {
      if (!cur.empty()) ::mkdir(cur.c_str(), 0755);
    }
    if (i < dir.size()) cur.push_back(dir[i]);
  }
  char tmp_suffix[64];
  std::snprintf(tmp_suffix, sizeof tmp_suffix, ".tmp.%d.%zu", static_cast<int>(::getpid()),
                std::hash<std::thread::id>()(std::this_thread::get_id()));
  const std::string tmp = path + tmp_suffix;
  FILE *f = std::fopen(tmp.c_str(), "wb");
  if (!f) return;
  // published only when every byte reached the file (a full disk fails at write, flush or close)
  bool ok = std::fwrite(code.data(), 1, code.size(), f) == code.size();
  ok = std::fflush(f) == 0 && ok;
  ok = ::fsync(::fileno(f)) == 0 && ok;
  ok = std::fclose(f) == 0 && ok;
  if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) std::remove(tmp.c_str());  // atomic publish
}

// hipRTC: source -> gfx950 code object (needs no device), through the disk cache
// *cached: the code came from the disk cache (whose entry a failed load then drops:
// cache_drop); no_cache_read: compile even if an entry exists.
bool compile(const std::string &src, std::vector<char> &code, std::string &err, std::string *cached = nullptr,
             bool no_cache_read = false) {
  // -O1/-O2 measured no faster to compile (the time is in the backend)
  const char *opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17"};
  const std::string dir = cache_dir();
  const std::string path = dir.empty() ? std::string() : cache_path(dir, src, opts, 3);
  if (cached) cached->clear();
  if (!path.empty() && !no_cache_read && cache_read(path, code)) {
    if (cached) *cached = path;
    g_disk_hits++;
    if (std::getenv("RS_AMD_JIT_VERBOSE")) std::fprintf(stderr, "[rs_amd jit] code-object cache hit %s\n", path.c_str());
    return true;
  }
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "rs_net.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
    err = "hiprtcCreateProgram failed";
    return false;
  }
  const hiprtcResult rc = hiprtcCompileProgram(prog, 3, opts);
  if (rc != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n, '\0');
    if (n) hiprtcGetProgramLog(prog, &log[0]);
    err = std::string("hiprtcCompileProgram: ") + hiprtcGetErrorString(rc) + "\n" + log.substr(0, 2000);
    hiprtcDestroyProgram(&prog);
    return false;
  }
  size_t code_size = 0;
  hiprtcGetCodeSize(prog, &code_size);
  code.resize(code_size);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  g_compiles++;
  if (code_size > 0 && !path.empty()) cache_write(dir, path, code);
  return code_size > 0;
}

}  // namespace

bool compile_check(const NetSpec &spec, std::string &err, double *ms, size_t *code_bytes) {
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<char> code;
  const Tuning tu = tuning();
  NetSpec sp = spec;  // RS_AMD_NET_CHECK_PIECES: check the 2 / 4-stripe small-shard variant
  const int cp = env_int("RS_AMD_NET_CHECK_PIECES", 1);  // 1, 2 or 4 (the layouts net_pieces() produces)
  sp.pieces = static_cast<uint32_t>(cp == 2 || cp == 4 ? cp : 1);
  const std::string name = kernel_name(sp, spec_key(sp, -1, tu)), src = generate_with(sp, name, tu);
  if (const char *dir = std::getenv("RS_AMD_JIT_DUMP")) {  // debug aid: keep the generated source
    if (FILE *f = std::fopen((std::string(dir) + "/" + name + ".hip").c_str(), "w")) {
      std::fputs(src.c_str(), f);
      std::fclose(f);
    }
  }
  const bool ok = compile(src, code, err);
  if (ms) *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (code_bytes) *code_bytes = code.size();
  return ok;
}

bool enabled() {
  const char *e = std::getenv("RS_AMD_JIT");
  return !(e && std::strcmp(e, "0") == 0);
}

namespace {

// set by the exit handler (Worker::push): a compile still in flight at process exit
// does not load its module
std::atomic<bool> g_exiting{false};

// source -> loaded module; no lock held (compiles run concurrently)
std::unique_ptr<Kernel> build_source(const std::string &name, const std::string &src, std::string &err) {
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<char> code;
  std::string cached;
  if (!compile(src, code, err, &cached)) return nullptr;
  if (g_exiting.load()) {
    err = "process exiting";
    return nullptr;
  }
  auto k = std::make_unique<Kernel>();
  hipError_t e = hipModuleLoadData(&k->module, code.data());
  if (e != hipSuccess && !cached.empty()) {  // a bad disk-cache entry: drop it, compile once more
    std::remove(cached.c_str());
    if (!compile(src, code, err, nullptr, true)) return nullptr;
    e = hipModuleLoadData(&k->module, code.data());
  }
  if (e != hipSuccess) {
    err = std::string("hipModuleLoadData: ") + hipGetErrorString(e);
    return nullptr;
  }
  e = hipModuleGetFunction(&k->fn, k->module, name.c_str());
  if (e != hipSuccess) {
    err = std::string("hipModuleGetFunction: ") + hipGetErrorString(e);
    return nullptr;
  }
  k->name = name;
  k->compile_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (std::getenv("RS_AMD_JIT_VERBOSE"))
    std::fprintf(stderr, "[rs_amd jit] %s compiled in %.0f ms (%zu B source, %zu B code)\n", name.c_str(),
                 k->compile_ms, src.size(), code.size());
  return k;
}

std::unique_ptr<Kernel> build(const NetSpec &spec, const std::string &key, const Tuning &tu, std::string &err) {
  const std::string name = kernel_name(spec, key);
  std::unique_ptr<Kernel> k = build_source(name, generate_with(spec, name, tu), err);
  if (!k) return nullptr;
  k->n_in = spec.n_in;
  k->n_out = spec.n_out;
  k->n_tiles = kernel_tiles(tu, spec);
  k->units = static_cast<uint32_t>(tu.units);
  k->pieces = spec.pieces;
  k->shared = shared_on(tu, spec);
  return k;
}

// Loaded modules are never unloaded (a launch may still use one); past
// RS_AMD_JIT_CACHE_MAX of them (default 1024) new maps run on their table kernels.
size_t module_cap() {
  const char *e = std::getenv("RS_AMD_JIT_CACHE_MAX");
  return e && *e ? static_cast<size_t>(std::max(0, std::atoi(e))) : 1024u;
}
const char *kCapErr = "module cache full (RS_AMD_JIT_CACHE_MAX)";

const Kernel *insert(const std::string &key, std::unique_ptr<Kernel> k) {  // g_mu held
  auto it = g_cache.find(key);
  if (it != g_cache.end()) return it->second.get();  // another thread won the race
  const Kernel *out = k.get();
  g_cache.emplace(key, std::move(k));
  return out;
}

// One background worker compiles the queued maps in order. At exit it drops the queue
// and finishes only the compile in flight (without loading it). The first push
// registers an exit handler that does this: registered after the HIP runtime was
// initialised, it runs before the runtime's own teardown, so no worker thread is still
// inside hipRTC / HIP calls while the runtime and this library are torn down (a
// process that exited during a background compile used to crash in teardown). The
// worker is defined after the caches above, so it is destroyed (joined) before them.
struct Job {
  std::string key, name;
  std::function<std::string()> gen;  // the kernel source (generated on the worker)
  std::function<void(Kernel &)> fill;  // launch metadata of the built kernel
  int dev;
  std::function<void()> host;  // a host job instead of a compile (run_host_job)
};

struct Worker {
  std::thread th;
  std::deque<Job> queue;
  std::condition_variable wake;
  bool stop = false;

  void push(Job j) {  // g_mu held
    if (stop) {  // after the exit handler: nothing compiles any more (the caller keeps its table kernel)
      g_pending.erase(j.key);
      g_failed.emplace(j.key, "process exiting");
      return;
    }
    queue.push_back(std::move(j));
    if (!th.joinable()) {
      static std::once_flag once;
      std::call_once(once, [] { std::atexit(stop_at_exit); });
      th = std::thread([this] { run(); });
    }
    wake.notify_one();
  }
  static void stop_at_exit();
  void shutdown() {
    {
      std::lock_guard<std::mutex> lk(g_mu);
      stop = true;
      for (const Job &j : queue) g_pending.erase(j.key);
      queue.clear();
      g_cv.notify_all();
    }
    wake.notify_all();
    if (th.joinable()) th.join();
  }
  void run() {
    for (;;) {
      Job j;
      {
        std::unique_lock<std::mutex> lk(g_mu);
        wake.wait(lk, [this] { return stop || !queue.empty(); });
        if (stop) return;
        j = std::move(queue.front());
        queue.pop_front();
      }
      if (j.host) {  // host work on the worker (a plan build): no module to insert
        if (hipSetDevice(j.dev) == hipSuccess) {
          try {
            j.host();
          } catch (...) {  // the caller keeps what it had (the job was an improvement)
          }
        }
        std::lock_guard<std::mutex> lk(g_mu);
        g_pending.erase(j.key);
        g_cv.notify_all();
        continue;
      }
      std::string e;
      std::unique_ptr<Kernel> k;
      if (hipSetDevice(j.dev) == hipSuccess) {
        k = build_source(j.name, j.gen(), e);
        if (k && j.fill) j.fill(*k);
      } else {
        e = "hipSetDevice failed";
      }
      std::lock_guard<std::mutex> lk(g_mu);
      if (k) insert(j.key, std::move(k));
      else g_failed.emplace(j.key, e);
      g_pending.erase(j.key);
      g_cv.notify_all();
    }
  }
  ~Worker() { shutdown(); }
} g_worker;

void Worker::stop_at_exit() {
  g_exiting.store(true);
  g_worker.shutdown();
}

bool env_on(const char *name) {
  const char *e = std::getenv(name);
  return e && *e && std::strcmp(e, "0") != 0;
}

}  // namespace

bool run_host_job(const std::string &key, std::function<void()> fn) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  const std::string full = std::to_string(dev) + ":host:" + key;
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_pending.count(full)) return true;
  g_pending.insert(full);
  try {
    g_worker.push(Job{full, "", nullptr, nullptr, dev, std::move(fn)});
  } catch (const std::exception &) {
    g_pending.erase(full);
    return false;
  }
  return true;
}

uint64_t max_async_blocks() {
  const int v = env_int("RS_AMD_NET_ASYNC_BLOCKS", -1);
  return v >= 0 ? static_cast<uint64_t>(v) : kMaxAsyncBlocks;
}

bool supports_async(uint32_t n_in, uint32_t n_out, uint64_t shard_bytes) {
  const uint64_t blocks = static_cast<uint64_t>(n_in) * ((n_out + kTileOut - 1) / kTileOut);
  return n_in > 0 && n_out > 0 && n_out <= kMaxOut && blocks <= std::max(max_blocks(), max_async_blocks()) &&
         shard_ok(shard_bytes);
}

const Kernel *get(const NetSpec &spec, std::string &err) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    err = "hipGetDevice failed";
    return nullptr;
  }
  const Tuning tu = tuning();
  const std::string key = spec_key(spec, dev, tu);
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_cache.find(key);
    if (it != g_cache.end()) return it->second.get();
    if (g_cache.size() >= module_cap()) {
      err = kCapErr;
      return nullptr;
    }
  }
  std::unique_ptr<Kernel> k = build(spec, key, tu, err);
  if (!k) return nullptr;
  std::lock_guard<std::mutex> lk(g_mu);
  return insert(key, std::move(k));
}

const Kernel *get_async(const NetSpec &spec, std::string &err, bool &pending) {
  pending = false;
  if (env_on("RS_AMD_JIT_SYNC")) return get(spec, err);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    err = "hipGetDevice failed";
    return nullptr;
  }
  const Tuning tu = tuning();
  const std::string key = spec_key(spec, dev, tu);
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_cache.find(key);
  if (it != g_cache.end()) return it->second.get();
  auto f = g_failed.find(key);
  if (f != g_failed.end()) {
    err = f->second;
    return nullptr;
  }
  if (g_cache.size() >= module_cap()) {
    err = kCapErr;
    return nullptr;
  }
  pending = true;
  if (g_pending.count(key)) return nullptr;
  g_pending.insert(key);
  try {
    const std::string name = kernel_name(spec, key);
    g_worker.push(Job{key, name, [spec, name, tu] { return generate_with(spec, name, tu); },
                      [spec, tu](Kernel &k) {
                        k.n_in = spec.n_in;
                        k.n_out = spec.n_out;
                        k.n_tiles = kernel_tiles(tu, spec);
                        k.units = static_cast<uint32_t>(tu.units);
                        k.pieces = spec.pieces;
                        k.shared = shared_on(tu, spec);
                      },
                      dev});
  } catch (const std::exception &ex) {  // no worker thread: the table kernel stays in use
    g_pending.erase(key);
    g_failed.emplace(key, std::string("background compile unavailable: ") + ex.what());
    err = g_failed[key];
    pending = false;
  }
  return nullptr;
}

const Kernel *get_source(const std::string &key, const std::string &name, const std::function<std::string()> &gen,
                         bool async, std::string &err, bool &pending) {
  pending = false;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    err = "hipGetDevice failed";
    return nullptr;
  }
  const std::string full = std::to_string(dev) + ":src:" + key;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_cache.find(full);
    if (it != g_cache.end()) return it->second.get();
    auto f = g_failed.find(full);
    if (f != g_failed.end()) {
      err = f->second;
      return nullptr;
    }
    if (g_cache.size() >= module_cap()) {
      err = kCapErr;
      return nullptr;
    }
    if (async && !env_on("RS_AMD_JIT_SYNC")) {
      pending = true;
      if (g_pending.count(full)) return nullptr;
      g_pending.insert(full);
      try {
        g_worker.push(Job{full, name, gen, nullptr, dev});
      } catch (const std::exception &ex) {
        g_pending.erase(full);
        g_failed.emplace(full, std::string("background compile unavailable: ") + ex.what());
        err = g_failed[full];
        pending = false;
      }
      return nullptr;
    }
  }
  std::unique_ptr<Kernel> k = build_source(name, gen(), err);
  std::lock_guard<std::mutex> lk(g_mu);
  if (!k) {
    g_failed.emplace(full, err);
    return nullptr;
  }
  return insert(full, std::move(k));
}

bool compile_source_check(const std::string &src, std::string &err, double *ms, size_t *code_bytes) {
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<char> code;
  const bool ok = compile(src, code, err);
  if (ms) *ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (code_bytes) *code_bytes = code.size();
  return ok;
}

void compile_stats(uint64_t *compiles, uint64_t *disk_hits, uint64_t *modules) {
  if (compiles) *compiles = g_compiles.load();
  if (disk_hits) *disk_hits = g_disk_hits.load();
  if (modules) {
    std::lock_guard<std::mutex> lk(g_mu);
    *modules = g_cache.size();
  }
}

size_t pending_jobs() {
  std::lock_guard<std::mutex> lk(g_mu);
  return g_pending.size();
}

void wait_pending() {
  std::unique_lock<std::mutex> lk(g_mu);
  g_cv.wait(lk, [] { return g_pending.empty(); });
}

hipError_t launch(const Kernel &k, const uint8_t *buf0, uint64_t stride0, const uint8_t *buf1, uint64_t stride1,
                  uint8_t *out, uint64_t out_stride, uint64_t shard_bytes, uint64_t n_stripes, hipStream_t s,
                  const uint8_t *buf2, uint64_t stride2) {
  if (n_stripes == 0) return hipSuccess;
  if (k.pieces > 1 && shard_bytes * k.pieces != kUnitBytes) return hipErrorInvalidValue;  // wrong kernel for sb
  trace_launch(k.name.c_str());
  if (k.shared) {  // one workgroup of n_tiles waves per 4 KiB unit (generate_shared)
    const uint64_t units = shard_bytes / kUnitBytes;
    if (units == 0 || units > 0x7fffffffull || shard_bytes % kUnitBytes) return hipErrorInvalidValue;
    for (uint64_t s0 = 0; s0 < n_stripes; s0 += 65535) {
      const uint32_t gy = static_cast<uint32_t>(std::min<uint64_t>(65535, n_stripes - s0));
      const unsigned char *a0 = buf0, *a1 = buf1 ? buf1 : buf0, *a2 = buf2 ? buf2 : a1;
      unsigned char *o = out;
      uint64_t st0 = stride0, st1 = buf1 ? stride1 : stride0, so = out_stride, sb = shard_bytes, first = s0;
      uint64_t st2 = buf2 ? stride2 : st1, nst = n_stripes;
      void *args[] = {&a0, &st0, &a1, &st1, &o, &so, &sb, &first, &a2, &st2, &nst};
      hipError_t e = hipModuleLaunchKernel(k.fn, static_cast<uint32_t>(units), gy, 1, 64 * k.n_tiles, 1, 1, 0, s, args,
                                           nullptr);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  // small shards: one launch row whose wave units each span k.pieces stripes
  const uint64_t units = k.pieces > 1 ? (n_stripes + k.pieces - 1) / k.pieces : shard_bytes / kUnitBytes;
  const uint64_t per_block = 4ull * k.units;
  // unit groups padded to a multiple of 8 (one per XCD, see generate()); the padding
  // workgroups find no unit and exit
  const uint64_t groups = (units + per_block - 1) / per_block;
  const uint64_t gx64 = (k.n_tiles > 1 ? (groups + 7) / 8 * 8 : groups) * k.n_tiles;
  if (gx64 > 0x7fffffffull) return hipErrorInvalidValue;
  const uint32_t gx = static_cast<uint32_t>(gx64);
  const uint64_t row = k.pieces > 1 ? n_stripes : 65535;  // stripes per launch
  for (uint64_t s0 = 0; s0 < n_stripes; s0 += row) {
    const uint32_t gy = k.pieces > 1 ? 1u : static_cast<uint32_t>(std::min<uint64_t>(65535, n_stripes - s0));
    const unsigned char *a0 = buf0, *a1 = buf1 ? buf1 : buf0;
    unsigned char *o = out;
    const unsigned char *a2 = buf2 ? buf2 : a1;
    uint64_t st0 = stride0, st1 = buf1 ? stride1 : stride0, so = out_stride, sb = shard_bytes, first = s0;
    uint64_t st2 = buf2 ? stride2 : st1, nst = n_stripes;
    void *args[] = {&a0, &st0, &a1, &st1, &o, &so, &sb, &first, &a2, &st2, &nst};
    hipError_t e = hipModuleLaunchKernel(k.fn, gx, gy, 1, 256, 1, 1, 0, s, args, nullptr);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace jit
}  // namespace rs
