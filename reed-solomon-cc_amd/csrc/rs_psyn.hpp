// rs_psyn.hpp — reconstruct with a per-stripe erasure pattern through syndromes on
// a bit-sliced network (rs_jit.hpp representation), one kernel per code.
//
// For a systematic linear code with encode coefficients G[r][t] (root.zig:136-173,
// corrected multiply: a GF(2^16)-linear map), a stripe with erased originals E and
// present recovery rows R (|R| = e = |E|, the first e present) satisfies
//   s_r = p_r ^ sum_{t not in E} G[r][t] d_t = sum_{t in E} G[r][t] d_t,
// so x_E = A^-1 s_R with A = G[R][E]. The syndromes of every row are one fixed
// k -> m network of the code (erased inputs and absent rows read as zero through a
// zero-record buffer resource: no branch, no load), compiled once; only the e x e
// solve differs per stripe (A^-1 built on the GPU by k_psyn_plan). The network leaves
// the syndromes in polynomial coordinates (the Cantor -> polynomial basis change is
// folded into its rows), where multiplying by alpha is a plane rotation plus three
// XORs (field polynomial 0x1002D): x_j = sum_i c_i alpha^i s walks that chain once
// per syndrome and XORs 16 planes into x_j under a wave-uniform branch per set bit of
// c (polynomial form of A^-1[j][r]); the restored outputs go back to Cantor
// coordinates through one fixed 16 x 16 network each.
//
// This replaces the per-stripe e x k table matrices of the matrix path (40 table
// multiplies per column for RS(10,4), v_perm-bound) for codes with k <= kMaxK and
// m <= kMaxM; the reference evaluates the erasure locator per call
// (Generic.zig:200-215, root.zig:268-335).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "rs_jit.hpp"

namespace rs {
namespace psyn {

// syndrome accumulators: 16 m VGPRs; restored outputs: all min(k, m) at once (16 each)
// for m <= 4, one at a time for m in 5..8 (the syndromes stay in registers)
constexpr uint32_t kMaxM = 8;
constexpr uint32_t kMaxK = 256;  // erased-original mask words in the plan block

struct Spec {
  uint32_t k = 0, m = 0, flags = 0;
  std::vector<uint16_t> images;  // encode map: images[(t * m + r) * 16 + b] (rs_jit NetSpec layout)
  std::vector<uint16_t> cantor;  // the 16 Cantor basis elements in polynomial form (rs_gf.hpp)
};

// restored outputs a kernel computes per stripe (the plan's max_out)
inline uint32_t max_out(uint32_t k, uint32_t m) { return k < m ? k : m; }
// u32 words of one stripe's plan block (rs_internal.hpp launch_psyn_plan): ceil(k / 32)
// erased-original mask words, the R row mask, the outputs restored, then the coefficients
inline uint32_t mask_words(uint32_t k) { return (k + 31) / 32; }
inline uint32_t plan_dwords(uint32_t k, uint32_t m) { return mask_words(k) + 2 + m * max_out(k, m); }

bool supports(uint64_t k, uint64_t m, uint64_t shard_bytes);
std::string generate(const Spec &s, const std::string &name);
// nullptr with pending = true while a background compile runs (the caller takes another path)
const jit::Kernel *get(const Spec &s, std::string &err, bool &pending);
bool compile_check(const Spec &s, std::string &err, double *ms, size_t *code_bytes);

// orig [stripe][k][sb] (stride os_), rec [stripe][m][sb] (rs_), out [stripe][..][sb]
// (so_): stripe s writes plan[s][3] rows; plan [n][plan_dwords] on the device
hipError_t launch(const jit::Kernel &kn, const Spec &s, const uint8_t *orig, uint64_t os_, const uint8_t *rec,
                  uint64_t rs_, uint8_t *out, uint64_t so_, uint64_t sb, uint64_t n_stripes, const uint32_t *plan,
                  hipStream_t st);

// Wide codes (chunk 32 / 64, any e <= m <= 64; outputs in groups of kSolveMaxOut, one
// group per blockIdx.z, coefficient stride cs = 8 * groups): the
// syndromes come from the bit-sliced FFT kernel with per-stripe masks (fftnet::Spec::dyn:
// erased shards read as zero, only the rows R stored into a scratch), and one generic
// kernel solves x = A^-1 (rec[R] ^ scratch[R]) with the alpha chains above, a runtime
// loop over the e syndromes (plan from launch_wps_plan, header at word `hdr` of a
// stripe's plan_dw-word block).
constexpr uint32_t kSolveMaxOut = 8;
std::string generate_solve(const uint16_t *cantor, const std::string &name);
const jit::Kernel *get_solve(const uint16_t *cantor, std::string &err);
bool compile_check_solve(const uint16_t *cantor, std::string &err, double *ms, size_t *code_bytes);
// shared_plan: one plan block for every stripe (a batch with one erasure pattern)
hipError_t launch_solve(const jit::Kernel &kn, const uint8_t *rec, uint64_t rs_, const uint8_t *scratch, uint64_t ss,
                        uint8_t *out, uint64_t so_, uint64_t sb, uint64_t n_stripes, const uint32_t *plan,
                        uint32_t plan_dw, uint32_t hdr, uint32_t cs, hipStream_t st, bool shared_plan = false);

}  // namespace psyn
}  // namespace rs
