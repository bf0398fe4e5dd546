// rs_internal.hpp — launch interface between the host codec (rs_capi.cpp) and
// the HIP kernels (rs_kernels.hip). Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <vector>

#include "rs_gf.hpp"

namespace rs {

// Launch record (rs_last_kernels): every launcher below and every hipRTC launch notes
// the kernel it launched for the calling thread; a C-ABI compute entry point clears the
// record when it starts (TraceScope, outermost call only), so after the call the record
// lists what that call actually ran, in launch order (repeats collapsed).
void trace_launch(const char *name);
struct TraceScope {
  TraceScope();
  ~TraceScope();
};
const char *trace_text();

// Encode: data [stripe][k][sb] -> parity [stripe][m][sb].
// Table block: n_chunks x ifft_tab_count(chunk) (chunk j has skew_delta (j+1)*chunk),
// then fft_tab_count(chunk) (skew_delta 0).
struct EncodeArgs {
  const uint8_t *data;
  uint64_t data_stripe_stride;
  uint8_t *parity;
  uint64_t parity_stripe_stride;
  uint64_t shard_bytes;
  uint64_t n_stripes;
  const RsTab *tabs;
  uint32_t chunk;        // ceilPow2(m)
  uint32_t n_chunks;     // IFFT chunks actually folded (D2 may drop one)
  uint32_t trunc_first;  // truncation of chunk 0 = min(k, chunk)
  uint32_t trunc_last;   // truncation of the last chunk (chunk, or k % chunk)
  uint32_t m;            // FFT truncation = recovery_count
  uint32_t k;
  uint32_t tabs_per_chunk;  // ifft_tab_count(chunk)
  uint32_t work;            // Wenc = alignUp(k, chunk) (generic path scratch positions)
  uint8_t *scratch;      // generic path only: [stripe][Wenc][sb]
  uint64_t scratch_stripes;
  bool contig;           // lane layout (dev::load_sym): contiguous waves vs split halves
  const uint32_t *skip = nullptr;  // device bitmask of k bits: data shards read as zero (syndrome reconstruct)
  // low-rate generic encode: scratch regions per stripe (coefficients + one per recovery
  // chunk of a launch; 0 = 1 + n_chunks) and the first recovery chunk of the launch
  uint32_t regions = 0, chunk0 = 0;
};

// Reconstruct: positions per root.zig:199-229 (recovery at [0,m), originals at
// [chunk, chunk+k), W = ceilPow2(chunk+k)). Plan arrays (device, uniform):
//   pos_src[W]: -1 none, else shard index | kSrcRecovery for recovery shards
//   pos_dst[W]: -1, else the restored slot of a missing original
//   tab_pre[W]: multiply by exp[erasures[p]] (present positions)
//   tab_post[W]: multiply by exp[65535 - erasures[p]] (missing originals)
struct DecodeArgs {
  const uint8_t *orig;
  uint64_t orig_stripe_stride;
  const uint8_t *rec;
  uint64_t rec_stripe_stride;
  uint8_t *out;
  uint64_t out_stripe_stride;
  uint64_t shard_bytes;
  uint64_t n_stripes;
  const RsTab *tab_ifft;
  const RsTab *tab_fft;
  const RsTab *tab_pre;
  const RsTab *tab_post;
  const int32_t *pos_src;
  const int32_t *pos_dst;
  uint32_t work;   // W
  uint32_t trunc;  // chunk + k (IFFT truncation; the FFT's too unless trunc_fft is set)
  uint32_t trunc_fft = 0;  // low rate: FFT truncated to k (only positions [0, k) are read)
  uint8_t *scratch;  // generic path only: [stripe][decode_generic_rows][sb] (launch_decode_generic)
  uint64_t scratch_stripes;
  // matrix variant: restored[j] = XOR_i map_ij(in[i]) over n_in received shards
  // pos_src[0..n_in) = sources, tab_mat[i * n_out + j] = map_ij (GF(2)-linear)
  const RsTab *tab_mat;
  uint32_t n_in;
  uint32_t n_out;
  bool contig;  // lane layout (dev::load_sym)
  // per-stripe patterns: tab_pre/tab_post/pos_src/pos_dst advance by
  // s * pattern_stride entries for stripe s (0 = one plan for the batch)
  uint64_t pattern_stride;
  // syndrome reconstruct: an input flagged kSrcXorScratch is rec[idx] ^ xsrc[idx]
  // (xsrc = the encode of the received data, [stripe][m][shard_bytes])
  const uint8_t *xsrc = nullptr;
  uint64_t xsrc_stripe_stride = 0;
  // matrix kernel with per-stripe matrices (per-stripe erasure patterns): stripe s
  // uses tab_mat + s * mat_stride, pos_src + s * src_stride and restores nout[s]
  // outputs (the rest of its row is not written)
  uint64_t mat_stride = 0;
  uint64_t src_stride = 0;
  const int32_t *nout = nullptr;
};
constexpr int32_t kSrcXorScratch = 0x20000000;
constexpr int32_t kSrcRecovery = 0x40000000;
constexpr int32_t kSrcIndexMask = 0x00FFFFFF;

// Kernel variants: fused register-resident for small transforms, generic
// (per-lane column walk over an HBM scratch work buffer) otherwise.
enum class Variant { kRegister, kGeneric, kMatrix, kWaveSplit, kMatrixTiled };

struct KernelChoice {
  Variant variant;
  int size;  // chunk (encode) or W (decode) for register kernels
  int nv;    // dword pairs per lane
  const char *name;
  int prefetch = 2;  // matrix kernel: inputs in flight per lane
};

// max_nv: widest per-lane access (1, 2, 4 dword pairs) the pointer/stride alignment allows
KernelChoice choose_encode(uint64_t k, uint64_t m, uint64_t shard_bytes, int max_nv);
KernelChoice choose_decode(uint64_t k, uint64_t m, uint64_t shard_bytes, int max_nv);
// scratch positions per stripe of the generic reconstruct (W transform + the FFT's kept rows)
uint64_t decode_generic_rows(uint64_t W, uint64_t trunc, uint64_t trunc_fft);
KernelChoice choose_decode_w(uint64_t W, uint64_t shard_bytes, int max_nv);  // by transform size

// Low-rate encode (rs_gf.hpp scalar_encode_low): EncodeArgs with chunk = C = ceilPow2(k),
// k, m, n_chunks = recovery chunks ceil(m / C), tabs = ifft_tab_count(C) tables of
// IFFT(C, skew 0) then tabs_per_chunk = fft_tab_count(C) tables of FFT(C, skew (j+1)C) per
// recovery chunk j. Register kernel for C <= 32, else the scratch-walking generic kernel
// (scratch [stripe][2C][sb]).
KernelChoice choose_encode_low(uint64_t C, uint64_t shard_bytes, int max_nv);
// the phases of the column transforms (rs_kernels.hip xform_ph): sub-problems of n positions at
// distance 2^dlo_log, first table ti of the size's IFFT (inv) or FFT table list
struct XPhase {
  uint32_t n, dlo_log;
  uint64_t ti;
};
void xform_phases(uint64_t size, bool inv, std::vector<XPhase> &out);

hipError_t launch_encode_low(const KernelChoice &kc, const EncodeArgs &a, hipStream_t s);

// Low-rate reconstruct in block form (rs_lowrate.cpp, C = ceilPow2(k) >= 128): C-point
// transforms only. enc: originals (erased ones flagged in enc.skip), tabs = the low-rate
// encode's tables for chunks j < n_chunks (enc.m = m' = the last recovery row used + 1),
// scratch [stripe][low_block_rows(C, k)][sb]. dec: out / out_stripe_stride, tab_fft =
// FFT(C, skew 0), tab_post / pos_dst per position < C (the erased originals). Per block
// K = j + 1: syn_idx[jC + p] >= 0 for the recovery rows used, syn_tab[jC + p] their multiplier
// L_r sigma_K, tabs_i + j * ifft_tab_count(C) = IFFT(C, skew KC), gamma[j] and u[j] (host)
// the block's scalars.
struct LowBlockArgs {
  EncodeArgs enc;
  DecodeArgs dec;
  const uint8_t *rec;
  uint64_t rec_stripe_stride;
  const int32_t *syn_idx;
  const RsTab *syn_tab;
  const RsTab *tabs_i;
  const RsTab *gamma;
  const RsTab *gamma1;  // 1 + gamma[j] (the whole-derivative scheme's W)
  const uint8_t *u;
  const uint8_t *used;  // host, per block: some recovery row of block K = j + 1 is read (else skipped)
};
uint64_t low_block_rows(uint64_t C, uint64_t k);
hipError_t launch_low_blocks(const LowBlockArgs &a, hipStream_t s);

// reconstruct as an n_out x n_in matrix of GF(2)-linear maps (decode matrix + GF MAC)
KernelChoice choose_decode_matrix(uint32_t n_out, uint64_t shard_bytes, int max_nv);
constexpr uint32_t kMatrixMaxOut = 8;
// output-tiled matrix kernel: 4 waves x kMtileEW outputs
constexpr int kMtileEW = 16;
constexpr uint32_t kMtileMaxOut = 4 * kMtileEW;
KernelChoice choose_decode_mtile(uint32_t n_out, uint64_t shard_bytes, int max_nv);

hipError_t launch_encode(const KernelChoice &kc, const EncodeArgs &a, hipStream_t s);
hipError_t launch_decode(const KernelChoice &kc, const DecodeArgs &a, hipStream_t s);

// contiguous lane layout possible for this shard size and lane width?
inline bool contig_ok(uint64_t shard_bytes, int nv) { return shard_bytes % (512ull * nv) == 0; }

// Device-side plans for per-stripe erasure patterns (W entries per stripe)
hipError_t launch_pattern_plan(const uint8_t *d_present, uint64_t present_stride, uint32_t k, uint32_t m, uint32_t C,
                               uint32_t W, uint64_t n, uint32_t max_e, bool d1, bool low, const uint16_t *d_exp,
                               const uint16_t *d_log, const uint16_t *d_log_walsh, uint16_t *logs, RsTab *pre,
                               RsTab *post, int32_t *src, int32_t *dst, int32_t *status, hipStream_t s);

// Per-stripe patterns as per-stripe e x k matrices (corrected multiply, W <= 32):
// images [n][k][max_e][16] (scratch), tabs [n][k][max_e] (matrix-kernel rows),
// srcs [n][k] (input shards), nout [n] (restored outputs per stripe)
hipError_t launch_pattern_matrix(const uint8_t *d_present, uint64_t present_stride, uint32_t k, uint32_t m, uint32_t C,
                                 uint32_t W, uint64_t n, uint32_t max_e, const uint16_t *logs, const RsTab *tab_ifft,
                                 const RsTab *tab_fft, const uint16_t *d_exp, const uint16_t *d_log, uint16_t *images,
                                 RsTab *tabs, int32_t *srcs, int32_t *nout, hipStream_t s);

// Per-stripe plan of the syndrome-network path (rs_psyn.hpp): G [m][k] encode
// coefficients then the 16 Cantor basis elements (polynomial form); plan
// [n][plan_dw] (k <= 256, m <= kPsynMaxM, max_out <= m; rs_psyn.hpp plan_dwords)
constexpr uint32_t kPsynMaxM = 8;
hipError_t launch_psyn_plan(const uint8_t *present, uint64_t present_stride, uint32_t k, uint32_t m, uint32_t max_out,
                            uint32_t max_e, uint64_t n, const uint16_t *G, const uint16_t *d_exp, const uint16_t *d_log,
                            uint32_t *plan, uint32_t plan_dw, int32_t *status, hipStream_t s);

// Per-stripe plan of the wide-code path: FFT mask block (dmw words) + solve header
// (rs_kernels.hip k_wps_plan / k_wps_plan_wave); plan_dw >= dmw + 2 + 64 + 64 * cs,
// cs = wps_coef_stride(max_e) (coefficients per syndrome: 8, or max_e rounded up to 8), m <= 64
uint32_t wps_coef_stride(uint32_t max_e);
hipError_t launch_wps_plan(const uint8_t *present, uint64_t present_stride, uint32_t k, uint32_t m, uint32_t max_e,
                           uint64_t n, const uint16_t *G, const uint16_t *d_exp, const uint16_t *d_log, uint32_t *plan,
                           uint32_t plan_dw, uint32_t dmw, int32_t *status, hipStream_t s);

// Per-stripe decode blocks of the fused FFT reconstruct (fftnet::Spec::decode; layout of
// fftnet::decode_block): trimmed [n][k+m] (scratch: the rows R = first e present
// recovery rows), logs [n][W] (scratch), blk [n][words]. FdecConsts: beta_K per data
// block (fftnet::decode_betas) and the (u|v) basis constants (rs_fftnet.cpp Basis::p).
struct FdecConsts {
  uint32_t beta[32];
  uint32_t p[8];
};
hipError_t launch_fdec_plan(const uint8_t *present, uint64_t present_stride, uint32_t k, uint32_t m, uint32_t C,
                            uint32_t W, uint64_t n, uint32_t max_e, const uint16_t *d_exp, const uint16_t *d_log,
                            const uint16_t *d_log_walsh, uint8_t *trimmed, uint16_t *logs, uint32_t *blk,
                            uint32_t dwm, uint32_t mko, uint32_t words, const FdecConsts &cst, int32_t *status,
                            hipStream_t s);

// present rows trimmed to the k shards the matrix path decodes from (out: [n][k+m])
hipError_t launch_trim_present(const uint8_t *present, uint64_t present_stride, uint32_t k, uint32_t m, uint64_t n,
                               uint8_t *out, hipStream_t s);

// Shard tails: pack one shard's last partial chunk into / out of the padded layout
hipError_t launch_tail_pack(const uint8_t *src, uint64_t src_stripe_stride, uint8_t *dst, uint64_t dst_stripe_stride,
                            uint64_t sb, uint64_t n, bool unpack, hipStream_t s);

// Engine shims (generic, in place on a single-stripe work buffer)
hipError_t launch_engine_fft(uint8_t *work, uint64_t shard_bytes, uint64_t pos, uint64_t size, uint64_t trunc,
                             const RsTab *tabs, bool inverse, hipStream_t s);
hipError_t launch_mul_scalar(uint8_t *chunks, uint64_t bytes, const RsTab *tab, hipStream_t s);

}  // namespace rs
