// rs_psyn.cpp — generator of the per-stripe syndrome-network reconstruct (rs_psyn.hpp).
#include "rs_psyn.hpp"

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <sstream>
#include <utility>

#include "rs_internal.hpp"

namespace rs {
namespace psyn {

bool supports(uint64_t k, uint64_t m, uint64_t shard_bytes) {
  return k >= 1 && k <= kMaxK && m >= 1 && m <= kMaxM && m <= kPsynMaxM && shard_bytes % jit::kUnitBytes == 0 &&
         shard_bytes > 0 && k * shard_bytes < 0x80000000ull && m * shard_bytes < 0x80000000ull;
}

namespace {

// code-shape knobs (part of the cache key): inputs loaded ahead, occupancy hint
// code shape (measured, profiles/r02/patterns_psyn*.jsonl): inputs loaded 2 ahead, an
// occupancy hint of 3 waves per SIMD, erased inputs skip their transform and network
// (5.0-5.15 -> 4.67 ms on RS(10,4) 1 MiB x 2048)
uint32_t prefetch() { return 2; }
int waves() { return 3; }
bool skip_erased() { return true; }

std::string key_of(const Spec &s) {
  std::string k = "psyn2:p" + std::to_string(prefetch()) + "w" + std::to_string(waves()) + "s" +
                  std::to_string(skip_erased()) + "v" + std::to_string(jit::net_vmask()) + ":" + std::to_string(s.k) +
                  ":" + std::to_string(s.m) + ":" + std::to_string(s.flags) + ":";
  k.append(reinterpret_cast<const char *>(s.images.data()), s.images.size() * sizeof(uint16_t));
  k.append(reinterpret_cast<const char *>(s.cantor.data()), s.cantor.size() * sizeof(uint16_t));
  return k;
}

std::string name_of(const Spec &s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : key_of(s)) h = (h ^ c) * 1099511628211ull;
  char name[96];
  std::snprintf(name, sizeof name, "rs_psyn_reconstruct_k%u_m%u_%016llx", s.k, s.m, static_cast<unsigned long long>(h));
  return name;
}

}  // namespace

namespace {
// rows of the Cantor <-> polynomial basis changes over bit-planes (rs_gf.hpp cantor_basis):
// to_poly[c] = mask of Cantor planes feeding polynomial plane c; to_cantor its inverse
void basis_rows(const uint16_t *cantor, uint16_t *to_poly, uint16_t *to_cantor) {
  for (int c = 0; c < 16; c++) to_poly[c] = 0;
  for (int i = 0; i < 16; i++)
    for (int c = 0; c < 16; c++)
      if (cantor[i] >> c & 1) to_poly[c] |= static_cast<uint16_t>(1u << i);
  uint32_t aug[16];
  for (int c = 0; c < 16; c++) aug[c] = to_poly[c] | (1u << (16 + c));
  for (int col = 0; col < 16; col++) {
    int piv = col;
    while (!(aug[piv] >> col & 1)) piv++;
    std::swap(aug[piv], aug[col]);
    for (int r = 0; r < 16; r++)
      if (r != col && (aug[r] >> col & 1)) aug[r] ^= aug[col];
  }
  for (int c = 0; c < 16; c++) to_cantor[c] = static_cast<uint16_t>(aug[c] >> 16);
}

// x_j ^= c * X for a polynomial-form coefficient held in `cf` (X0..X15 = the input's
// polynomial planes, consumed): the alpha chain with one uniform branch per set bit
void emit_chain(std::ostringstream &o, uint32_t j) {
  std::vector<int> nm(16);
  for (int c = 0; c < 16; c++) nm[c] = c;
  for (int i = 0; i < 16; i++) {
    o << "  if ((cf >> " << i << ") & 1u) {";
    for (int c = 0; c < 16; c++) o << " x" << j << "_" << c << " ^= X" << nm[c] << ";";
    o << " }\n";
    if (i == 15) break;
    const int top = nm[15];
    for (int c = 15; c > 0; c--) nm[c] = nm[c - 1];
    nm[0] = top;
    o << "  X" << nm[2] << " ^= X" << top << "; X" << nm[3] << " ^= X" << top << "; X" << nm[5] << " ^= X" << top << ";\n";
  }
}
}  // namespace

std::string generate(const Spec &s, const std::string &name) {
  const uint32_t K = s.k, M = s.m, MO = max_out(s.k, s.m), PDW = plan_dwords(s.k, s.m), NW = mask_words(s.k);
  std::ostringstream o;
  // non-temporal loads and stores (every byte is touched once)
  o << "#define RS_NT 3\n" << jit::net_prelude();
  o << "#define LDB(r, vo, so) __builtin_amdgcn_raw_buffer_load_b128((r), (vo), (so), 2)\n"
       "__device__ __forceinline__ Raw ldb(__amdgpu_buffer_rsrc_t r, u32 vo, u32 so) {\n"
       "  Raw x;\n  x.a0 = LDB(r, vo, so);\n  x.a1 = LDB(r, vo + 1024u, so);\n"
       "  x.b0 = LDB(r, vo + 2048u, so);\n  x.b1 = LDB(r, vo + 3072u, so);\n  return x;\n}\n";
  o << "extern \"C\" __global__ __launch_bounds__(256) ";
  // occupancy hint: 3 waves / SIMD for m <= 4 (168 VGPRs); 2 above (the 16 m syndrome
  // planes stay live through the solve: a 3-wave cap spills ~2,900 VGPRs for RS(32,8))
  const int wv = M <= 4 ? waves() : std::min(waves(), 2);
  if (wv) o << "__attribute__((amdgpu_waves_per_eu(" << wv << ", 8))) ";
  o << "void " << name
    << "(const unsigned char *__restrict__ b0, u64 s0, const unsigned char *__restrict__ b1, u64 s1,\n"
       "    unsigned char *__restrict__ out, u64 so, u64 sb, u64 stripe0, const u32 *__restrict__ plan) {\n"
       "  const u32 lane = threadIdx.x & 63u, ll = lane & 31u;\n"
       "  const u64 s = stripe0 + blockIdx.y;\n"
       "  const u64 unit = (u64)blockIdx.x * 4u + (threadIdx.x >> 6);\n"
       "  if (unit * 4096u >= sb) return;\n"
    << "  const u32 *pl = plan + s * " << PDW << "u;\n"
    << "  const u32 ne = pl[" << NW + 1 << "];\n"
       "  if (ne == 0u) return;\n"
    << "  const u32 rm = pl[" << NW << "], sbl = (u32)sb;\n";
  for (uint32_t w = 0; w < NW; w++) o << "  const u32 em" << w << " = pl[" << w << "];\n";
  o <<
       "  const u32 off = (u32)unit * 4096u + (ll >> 1) * 64u + (lane >= 32u ? 32u : 0u) + (ll & 1u) * 16u;\n"
       "  const __amdgpu_buffer_rsrc_t RZ = __builtin_amdgcn_make_buffer_rsrc((void *)b0, (short)0, 0, 0x00020000);\n"
    << "  const __amdgpu_buffer_rsrc_t RD = __builtin_amdgcn_make_buffer_rsrc((void *)(b0 + s * s0), (short)0, (int)("
    << K << "u * sbl), 0x00020000);\n"
    << "  const __amdgpu_buffer_rsrc_t RR = __builtin_amdgcn_make_buffer_rsrc((void *)(b1 + s * s1), (short)0, (int)("
    << M << "u * sbl), 0x00020000);\n"
    << "  unsigned char *O = out + s * so;\n";
  // syndromes s_r = p_r ^ Enc_r(data with E read as zero): the code's fixed network,
  // its rows composed with the Cantor -> polynomial basis change (poly bit c of a
  // symbol = XOR of its Cantor bits i with bit c of cantor[i])
  uint16_t to_poly[16], to_cantor[16];
  basis_rows(s.cantor.data(), to_poly, to_cantor);
  auto compose = [&](const std::vector<uint16_t> &rows) {  // rows over Cantor output planes -> poly
    std::vector<uint16_t> out(rows.size(), 0);
    for (size_t r = 0; r < rows.size() / 16; r++)
      for (int c = 0; c < 16; c++)
        for (int i = 0; i < 16; i++)
          if (to_poly[c] >> i & 1) out[r * 16 + c] ^= rows[r * 16 + i];
    return out;
  };
  const uint32_t n_acc = 16 * M;
  o << "  u32 ";
  for (uint32_t r = 0; r < n_acc; r++) o << "a" << r << " = 0u" << (r + 1 < n_acc ? ", " : ";\n");
  std::vector<bool> init(n_acc, true);
  // inputs: data 0..K-1, then recovery rows 0..M-1; input i + PF is loaded before input
  // i is transformed, and a scheduling barrier closes every input (otherwise the
  // compiler hoists every load to the top: 512 VGPRs and spills)
  const uint32_t n_inputs = K + M, PF = prefetch();
  auto load = [&](uint32_t i) {
    if (i >= n_inputs) return;
    o << "  const Raw R" << i << " = ";
    if (i < K)
      o << "ldb(((em" << i / 32 << " >> " << i % 32 << ") & 1u) ? RZ : RD, off, " << i << "u * sbl);\n";
    else
      o << "ldb(((rm >> " << i - K << ") & 1u) ? RR : RZ, off, " << i - K << "u * sbl);\n";
  };
  for (uint32_t i = 0; i < PF; i++) load(i);
  for (uint32_t i = 0; i < n_inputs; i++) {
    load(i + PF);
    // an erased input (read as zeros) skips its transform and network
    // under a wave-uniform branch; its load stays unconditional (prefetch order)
    if (skip_erased())
      o << "  if (!(" << (i < K ? "(em" + std::to_string(i / 32) + " >> " + std::to_string(i % 32) + ") & 1u"
                                : "!((rm >> " + std::to_string(i - K) + ") & 1u)")
        << "))";
    o << "  {\n  u32 P[16];\n  planes(R" << i << ", P);\n";
    std::vector<uint16_t> rows(n_acc, 0);
    if (i < K) {
      for (uint32_t r = 0; r < M; r++)
        for (int b = 0; b < 16; b++) {
          const uint16_t img = s.images[(static_cast<size_t>(i) * M + r) * 16 + b];
          for (int c = 0; c < 16; c++)
            if (img >> c & 1) rows[r * 16 + c] |= static_cast<uint16_t>(1u << b);
        }
    } else {
      for (int c = 0; c < 16; c++) rows[(i - K) * 16 + c] = static_cast<uint16_t>(1u << c);  // p_r itself
    }
    jit::emit_network_input(o, compose(rows), init, static_cast<int>(i));
    o << "  }\n  __builtin_amdgcn_sched_barrier(0);\n";
  }
  // pinned: otherwise the compiler sinks the network's last XORs into the conditional
  // solve blocks below, keeping every input's Four-Russians terms live (512 VGPRs)
  for (uint32_t r = 0; r < n_acc; r++) o << "  asm volatile(\"\" : \"+v\"(a" << r << "));\n";
  // x_j = sum_{r in R} A^-1[j][i(r)] s_r in polynomial coordinates: per syndrome the
  // chain X = s_r * alpha^i (x^16 = x^5 + x^3 + x^2 + 1), XORed into x_j where bit i of
  // the stripe's coefficient is set (wave-uniform branches)
  auto store_out = [&](uint32_t j) {  // back to Cantor coordinates, then store
    o << "  {\n  u32 P[16] = {";
    for (int c = 0; c < 16; c++) o << "x" << j << "_" << c << (c == 15 ? "};\n" : ", ");
    o << "  u32 ";
    for (int c = 0; c < 16; c++) o << "z" << c << (c == 15 ? ";\n" : ", ");
    std::vector<uint16_t> rows(to_cantor, to_cantor + 16);
    std::vector<bool> oinit(16, false);
    std::ostringstream net;
    jit::emit_network_input(net, rows, oinit, static_cast<int>(1000 + j));
    std::string code = net.str();  // the network writes a<c>: rename to z<c> (the syndromes live on)
    for (int c = 15; c >= 0; c--) {
      const std::string from = "a" + std::to_string(c), to = "z" + std::to_string(c);
      for (size_t at = 0; (at = code.find(from, at)) != std::string::npos;) {
        const bool word_start = at == 0 || !(std::isalnum(static_cast<unsigned char>(code[at - 1])) || code[at - 1] == '_');
        const size_t end = at + from.size();
        const bool word_end = end >= code.size() || !std::isdigit(static_cast<unsigned char>(code[end]));
        if (word_start && word_end) {
          code.replace(at, from.size(), to);
          at += to.size();
        } else {
          at = end;
        }
      }
    }
    o << code;
    for (int c = 0; c < 16; c++)
      if (!oinit[c]) o << "  z" << c << " = 0u;\n";
    o << "  u32 Q[16] = {";
    for (int c = 0; c < 16; c++) o << "z" << c << (c == 15 ? "};\n" : ", ");
    o << "  st(O + " << j << "ull * sb + off, Q);\n  }\n";
  };
  if (M <= 4) {  // every output accumulates at once (16 MO + 16 M VGPRs)
    o << "  u32 ";
    for (uint32_t j = 0; j < MO; j++)
      for (int c = 0; c < 16; c++) o << "x" << j << "_" << c << " = 0u" << (j + 1 == MO && c == 15 ? ";\n" : ", ");
    for (uint32_t r = 0; r < M; r++) {
      o << "  if ((rm >> " << r << ") & 1u) {\n";
      for (uint32_t j = 0; j < MO; j++) {
        // one chain per (r, j): branches on one coefficient only (branches on several
        // correlated conditions let the compiler thread and duplicate blocks)
        o << "  if (" << j << "u < ne) {\n  const u32 cf = pl[" << NW + 2 + r * MO + j << "];\n  u32 ";
        for (int c = 0; c < 16; c++) o << "X" << c << " = a" << r * 16 + c << (c == 15 ? ";\n" : ", ");
        emit_chain(o, j);
        o << "  }\n";
      }
      o << "  }\n  __builtin_amdgcn_sched_barrier(0);\n";
    }
    for (uint32_t j = 0; j < MO; j++) {
      o << "  if (" << j << "u < ne)\n";
      store_out(j);
    }
  } else {  // m in 5..8: one output at a time (16 M + 32 VGPRs for the solve)
    for (uint32_t j = 0; j < MO; j++) {
      o << "  if (" << j << "u < ne) {\n  u32 ";
      for (int c = 0; c < 16; c++) o << "x" << j << "_" << c << " = 0u" << (c == 15 ? ";\n" : ", ");
      for (uint32_t r = 0; r < M; r++) {
        o << "  if ((rm >> " << r << ") & 1u) {\n  const u32 cf = pl[" << NW + 2 + r * MO + j << "];\n  u32 ";
        for (int c = 0; c < 16; c++) o << "X" << c << " = a" << r * 16 + c << (c == 15 ? ";\n" : ", ");
        emit_chain(o, j);
        o << "  }\n";
      }
      store_out(j);
      o << "  }\n  __builtin_amdgcn_sched_barrier(0);\n";
    }
  }
  o << "}\n";
  return o.str();
}


// The wide-code solve (rs_psyn.hpp launch_solve): one generic kernel, all codes.
std::string generate_solve(const uint16_t *cantor, const std::string &name) {
  uint16_t to_poly[16], to_cantor[16];
  basis_rows(cantor, to_poly, to_cantor);
  constexpr uint32_t MO = kSolveMaxOut;
  std::ostringstream o;
  o << "#define RS_NT 3\n" << jit::net_prelude();
  o << "extern \"C\" __global__ __launch_bounds__(256) void " << name
    << "(const unsigned char *__restrict__ rec, u64 rs, const unsigned char *__restrict__ scr, u64 ss,\n"
       "    unsigned char *__restrict__ out, u64 so, u64 sb, u64 stripe0, const u32 *__restrict__ plan, u32 pw, u32 hdr,\n"
       "    u32 cs) {\n"
       "  const u32 lane = threadIdx.x & 63u, ll = lane & 31u;\n"
       "  const u64 s = stripe0 + blockIdx.y;\n"
       "  const u64 unit = (u64)blockIdx.x * 4u + (threadIdx.x >> 6);\n"
       "  if (unit * 4096u >= sb) return;\n"
       "  const u32 *pl = plan + s * pw + hdr;\n"
       // output group blockIdx.z: originals g8 .. g8 + 7 of the stripe's erased list
       "  const u32 g8 = blockIdx.z * " << MO << "u, e = pl[1];\n"
       "  if (pl[0] <= g8) return;\n"
       "  const u32 ne = pl[0] - g8;\n"
       "  const u32 off = (u32)unit * 4096u + (ll >> 1) * 64u + (lane >= 32u ? 32u : 0u) + (ll & 1u) * 16u;\n"
       "  const unsigned char *RB = rec + s * rs, *SB = scr + s * ss;\n"
       "  unsigned char *O = out + s * so;\n";
  o << "  u32 ";
  for (uint32_t j = 0; j < MO; j++)
    for (int c = 0; c < 16; c++) o << "x" << j << "_" << c << " = 0u" << (j + 1 == MO && c == 15 ? ";\n" : ", ");
  // syndrome i = rec[R_i] ^ scratch[R_i]; the next one is loaded during this one's work
  o << "  Raw Rc = ldx(RB + (u64)pl[2] * sb + off, SB + (u64)pl[2] * sb + off);\n"
       "#pragma unroll 1\n"
       "  for (u32 i = 0; i < e; i++) {\n"
       "  Raw Rn = Rc;\n"
       "  if (i + 1u < e) { const u64 r = pl[3u + i]; Rn = ldx(RB + r * sb + off, SB + r * sb + off); }\n"
       "  u32 P[16];\n  planes(Rc, P);\n  u32 ";
  for (int c = 0; c < 16; c++) o << "a" << c << (c == 15 ? ";\n" : ", ");
  {
    std::vector<uint16_t> rows(to_poly, to_poly + 16);
    std::vector<bool> init(16, false);
    jit::emit_network_input(o, rows, init, 900);
    for (int c = 0; c < 16; c++)
      if (!init[c]) o << "  a" << c << " = 0u;\n";
  }
  // one alpha chain per syndrome shared by the group's outputs: step i XORs s * alpha^i
  // into every output whose coefficient has bit i (the chain's 45 XORs once, not per output)
  o << "  const u32 *cfp = pl + " << 2 + 64 << "u + i * cs + g8;\n";
  for (uint32_t j = 0; j < MO; j++) o << "  const u32 cf" << j << " = " << j << "u < ne ? cfp[" << j << "] : 0u;\n";
  o << "  u32 ";
  for (int c = 0; c < 16; c++) o << "X" << c << " = a" << c << (c == 15 ? ";\n" : ", ");
  {
    std::vector<int> nm(16);
    for (int c = 0; c < 16; c++) nm[c] = c;
    for (int i = 0; i < 16; i++) {
      for (uint32_t j = 0; j < MO; j++) {
        o << "  if ((cf" << j << " >> " << i << ") & 1u) {";
        for (int c = 0; c < 16; c++) o << " x" << j << "_" << c << " ^= X" << nm[c] << ";";
        o << " }\n";
      }
      if (i == 15) break;
      const int top = nm[15];
      for (int c = 15; c > 0; c--) nm[c] = nm[c - 1];
      nm[0] = top;
      o << "  X" << nm[2] << " ^= X" << top << "; X" << nm[3] << " ^= X" << top << "; X" << nm[5] << " ^= X" << top << ";\n";
    }
  }
  o << "  Rc = Rn;\n  }\n";
  for (uint32_t j = 0; j < MO; j++) {
    o << "  if (" << j << "u < ne) {\n  u32 P[16] = {";
    for (int c = 0; c < 16; c++) o << "x" << j << "_" << c << (c == 15 ? "};\n" : ", ");
    o << "  u32 ";
    for (int c = 0; c < 16; c++) o << "a" << c << (c == 15 ? ";\n" : ", ");
    std::vector<uint16_t> rows(to_cantor, to_cantor + 16);
    std::vector<bool> init(16, false);
    jit::emit_network_input(o, rows, init, static_cast<int>(1000 + j));
    for (int c = 0; c < 16; c++)
      if (!init[c]) o << "  a" << c << " = 0u;\n";
    o << "  u32 Q[16] = {";
    for (int c = 0; c < 16; c++) o << "a" << c << (c == 15 ? "};\n" : ", ");
    o << "  st(O + (u64)(g8 + " << j << "u) * sb + off, Q);\n  }\n";
  }
  o << "}\n";
  return o.str();
}

const jit::Kernel *get_solve(const uint16_t *cantor, std::string &err) {
  // v3: output groups (blockIdx.z), one alpha chain per syndrome
  std::string key = "psolve:v3:o" + std::to_string(kSolveMaxOut) + "v" + std::to_string(jit::net_vmask()) + ":";
  key.append(reinterpret_cast<const char *>(cantor), 16 * sizeof(uint16_t));
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : key) h = (h ^ c) * 1099511628211ull;
  char name[64];
  std::snprintf(name, sizeof name, "rs_psyn_solve_o%u_%016llx", kSolveMaxOut, static_cast<unsigned long long>(h));
  const std::string nm = name;
  std::vector<uint16_t> cb(cantor, cantor + 16);
  bool pending = false;
  return jit::get_source(key, nm, [cb, nm] { return generate_solve(cb.data(), nm); }, false, err, pending);
}

bool compile_check_solve(const uint16_t *cantor, std::string &err, double *ms, size_t *code_bytes) {
  const std::string src = generate_solve(cantor, "rs_psyn_solve_check");
  if (const char *dir = std::getenv("RS_AMD_JIT_DUMP")) {
    if (FILE *f = std::fopen((std::string(dir) + "/rs_psyn_solve_check.hip").c_str(), "w")) {
      std::fputs(src.c_str(), f);
      std::fclose(f);
    }
  }
  return jit::compile_source_check(src, err, ms, code_bytes);
}

hipError_t launch_solve(const jit::Kernel &kn, const uint8_t *rec, uint64_t rs_, const uint8_t *scratch, uint64_t ss,
                        uint8_t *out, uint64_t so_, uint64_t sb, uint64_t n_stripes, const uint32_t *plan,
                        uint32_t plan_dw, uint32_t hdr, uint32_t cs, hipStream_t st, bool shared_plan) {
  if (n_stripes == 0) return hipSuccess;
  if (sb == 0 || sb % jit::kUnitBytes || sb >= (1ull << 32)) return hipErrorInvalidValue;
  if (cs == 0 || cs % kSolveMaxOut || cs > 64 || plan_dw < hdr + 2 + 64 + 64 * cs) return hipErrorInvalidValue;
  const uint32_t groups = cs / kSolveMaxOut;
  const uint64_t gx = (sb / jit::kUnitBytes + 3) / 4;
  trace_launch(kn.name.c_str());
  for (uint64_t s0 = 0; s0 < n_stripes; s0 += 65535) {
    const uint32_t gy = static_cast<uint32_t>(std::min<uint64_t>(65535, n_stripes - s0));
    const unsigned char *a0 = rec, *a1 = scratch;
    unsigned char *o = out;
    uint64_t st0 = rs_, st1 = ss, so = so_, sbv = sb, first = s0;
    const uint32_t *pp = plan;
    uint32_t pw = shared_plan ? 0u : plan_dw, hd = hdr, c = cs;  // pw: the kernel's per-stripe plan stride
    void *args[] = {&a0, &st0, &a1, &st1, &o, &so, &sbv, &first, &pp, &pw, &hd, &c};
    hipError_t e = hipModuleLaunchKernel(kn.fn, static_cast<uint32_t>(gx), gy, groups, 256, 1, 1, 0, st, args, nullptr);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

const jit::Kernel *get(const Spec &s, std::string &err, bool &pending) {
  const std::string name = name_of(s);
  // small kernels (RS(10,4): ~2 s of hipRTC) compile in the call; larger ones (RS(32,8):
  // ~8 s) in the background while the caller takes its next path
  const bool async = static_cast<uint64_t>(s.k + s.m) * ((s.m + 3) / 4) > 64;
  return jit::get_source(key_of(s), name, [s, name] { return generate(s, name); }, async, err, pending);
}

bool compile_check(const Spec &s, std::string &err, double *ms, size_t *code_bytes) {
  const std::string name = name_of(s);
  const std::string src = generate(s, name);
  if (const char *dir = std::getenv("RS_AMD_JIT_DUMP")) {
    if (FILE *f = std::fopen((std::string(dir) + "/" + name + ".hip").c_str(), "w")) {
      std::fputs(src.c_str(), f);
      std::fclose(f);
    }
  }
  return jit::compile_source_check(src, err, ms, code_bytes);
}

hipError_t launch(const jit::Kernel &kn, const Spec &s, const uint8_t *orig, uint64_t os_, const uint8_t *rec,
                  uint64_t rs_, uint8_t *out, uint64_t so_, uint64_t sb, uint64_t n_stripes, const uint32_t *plan,
                  hipStream_t st) {
  if (n_stripes == 0) return hipSuccess;
  if (!supports(s.k, s.m, sb)) return hipErrorInvalidValue;
  const uint64_t units = sb / jit::kUnitBytes, gx = (units + 3) / 4;
  if (gx > 0x7fffffffull) return hipErrorInvalidValue;
  trace_launch(kn.name.c_str());
  for (uint64_t s0 = 0; s0 < n_stripes; s0 += 65535) {
    const uint32_t gy = static_cast<uint32_t>(std::min<uint64_t>(65535, n_stripes - s0));
    const unsigned char *a0 = orig, *a1 = rec;
    unsigned char *o = out;
    uint64_t st0 = os_, st1 = rs_, so = so_, sbv = sb, first = s0;
    const uint32_t *pp = plan;
    void *args[] = {&a0, &st0, &a1, &st1, &o, &so, &sbv, &first, &pp};
    hipError_t e = hipModuleLaunchKernel(kn.fn, static_cast<uint32_t>(gx), gy, 1, 256, 1, 1, 0, st, args, nullptr);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace psyn
}  // namespace rs
