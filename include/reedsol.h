/*
 * reedsol.h — C ABI of the MI355X-native Reed-Solomon engine (librs_amd.so).
 *
 * Drop-in for the encode/decode path of usebeforefree/reed-solomon-cc
 * (Zig, snapshot 2025-12-12): systematic RS over GF(2^16) in a Cantor basis,
 * Lin-Chung-Han additive FFT, "high rate" codec. Every entry point cites the
 * reference interface it replaces (paths relative to the reference repo).
 * Plain pointers and sizes only; no HIP or torch types in any signature
 * (a stream is passed as an opaque `void*`, i.e. a hipStream_t or NULL).
 *
 * Shard layout: the reference's own — a shard of shard_bytes is L =
 * shard_bytes/64 chunks of 64 B; in a chunk, bytes [0,32) are the low bytes
 * and [32,64) the high bytes of 32 GF(2^16) symbols (Generic.zig:152-156,
 * root.zig:373-383). No transposition anywhere.
 *
 * Every function returns an rs_status; none aborts. Results are bit-exact
 * with the reference algorithm (RS_FLAG_REF_LITERAL reproduces its two
 * arithmetic/schedule defects D1/D2).
 */
#ifndef REEDSOL_AMD_H
#define REEDSOL_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Status codes. 1..11 mirror the Zig error set of root.zig
 * (TooFewOriginalShards .. Overflow); 12.. are conditions where the
 * reference panics or that only a device engine can hit. */
typedef enum rs_status {
  RS_OK = 0,
  RS_ERR_TOO_FEW_ORIGINAL_SHARDS = 1,  /* root.zig:20, 139 */
  RS_ERR_NOT_ENOUGH_SHARDS = 2,        /* root.zig:58, 272 */
  RS_ERR_INVALID_SHARD_SIZE = 3,       /* root.zig:103, 201 */
  RS_ERR_UNSUPPORTED_SHARD_COUNT = 4,  /* root.zig:398, 407 */
  RS_ERR_TOO_MANY_ORIGINAL_SHARDS = 5, /* root.zig:129 */
  RS_ERR_DIFFERENT_SHARD_SIZE = 6,     /* root.zig:130, 243, 259 */
  RS_ERR_INVALID_SHARD_INDEX = 7,      /* root.zig:240, 254 */
  RS_ERR_DUPLICATE_SHARD_INDEX = 8,    /* root.zig:241, 256 */
  RS_ERR_TOO_MANY_SHARDS = 9,          /* root.zig:242, 258 */
  RS_ERR_OUT_OF_MEMORY = 10,           /* allocator failure */
  RS_ERR_OVERFLOW = 11,                /* std.math.ceilPowerOfTwo */
  RS_ERR_LOW_RATE_UNSUPPORTED = 12,    /* root.zig:120, 227 @panic("TODO"); no longer returned (every path serves low-rate codes) */
  RS_ERR_SHARD_TAIL_UNSUPPORTED = 13,  /* root.zig:385 @panic("TODO"); no longer returned (tails are coded) */
  RS_ERR_INVALID_ARGUMENT = 14,        /* NULL pointer / bad stride */
  RS_ERR_DEVICE = 15,                  /* HIP runtime error (message: rs_last_error()) */
  RS_ERR_NO_DEVICE = 16,               /* no gfx950 device visible */
} rs_status;

/* flags for the *_dev and engine entry points */
#define RS_FLAG_CORRECTED 0u
#define RS_FLAG_QUIRK_D1 1u /* Generic.zig:283: t1_hi used for nibble 0 of the hi product */
#define RS_FLAG_QUIRK_D2 2u /* root.zig:151: `<` drops the last full chunk when k % chunk == 0 */
#define RS_FLAG_REF_LITERAL (RS_FLAG_QUIRK_D1 | RS_FLAG_QUIRK_D2)

typedef void *rs_stream_t; /* hipStream_t, or NULL for the default stream */

/* ------------------------------------------------------------------ info */
const char *rs_version(void);
const char *rs_status_name(int status);  /* "NotEnoughShards", ... (Zig error names) */
const char *rs_last_error(void);         /* thread-local detail for the last non-OK status */
/* root.zig:397-415 useHighRate: 1 high rate, 0 low rate, negative = -rs_status */
int rs_use_high_rate(uint64_t original_count, uint64_t recovery_count);

/* ------------------------------------------- one-shot host API (root.zig:14-84)
 * Host buffers in, host buffers out; internally H2D -> fused HIP kernel -> D2H.
 * Generalises the reference's 64-byte-typed result to any even shard_bytes
 * (defect D6); a tail of shard_bytes % 64 bytes is coded as one more chunk in the
 * layout undoLastChunkEncoding implies (root.zig:338-348; the reference itself
 * panics on tails, root.zig:385). Caller owns every buffer. */

/* replaces `encode(allocator, original_count, recovery_count, original)` root.zig:14-30.
 * original[k] -> recovery_out[m] (each shard_bytes). */
int rs_encode(uint64_t original_count, uint64_t recovery_count, size_t shard_bytes,
              const uint8_t *const *original, uint8_t *const *recovery_out);

/* replaces `decode(allocator, original_count, recovery_count, original, recovery)` root.zig:32-84.
 * original[i] / recovery[i] == NULL marks a missing shard. restored_out[k]
 * receives every original (present ones copied through, root.zig:76-81). */
int rs_decode(uint64_t original_count, uint64_t recovery_count, size_t shard_bytes,
              const uint8_t *const *original, const uint8_t *const *recovery, uint8_t *const *restored_out);

/* ----------------------------------------- Encoder object (root.zig:86-174) */
typedef struct rs_encoder rs_encoder;
/* Encoder.init root.zig:94-122 */
int rs_encoder_new(uint64_t original_count, uint64_t recovery_count, size_t shard_bytes, rs_encoder **out);
/* Encoder.addOriginalShard root.zig:128-134 */
int rs_encoder_add_original_shard(rs_encoder *enc, const uint8_t *shard, size_t len);
/* Encoder.encode root.zig:136-173: recovery_out[m] receives borrowed pointers
 * valid until the next encode / rs_encoder_free. */
int rs_encoder_encode(rs_encoder *enc, const uint8_t **recovery_out);
/* Encoder.deinit root.zig:124-126 (resets for reuse: rs_encoder_reset) */
void rs_encoder_free(rs_encoder *enc);
int rs_encoder_reset(rs_encoder *enc);

/* ----------------------------------------- Decoder object (root.zig:176-336)
 * The reference keeps these methods private; exposed here with the same checks. */
typedef struct rs_decoder rs_decoder;
int rs_decoder_new(uint64_t original_count, uint64_t recovery_count, size_t shard_bytes, rs_decoder **out);
int rs_decoder_add_original_shard(rs_decoder *dec, uint64_t index, const uint8_t *shard, size_t len);
int rs_decoder_add_recovery_shard(rs_decoder *dec, uint64_t index, const uint8_t *shard, size_t len);
/* restored_out[k]: borrowed pointers to all k originals (supplied ones copied,
 * missing ones restored), valid until the next decode / rs_decoder_free. */
int rs_decoder_decode(rs_decoder *dec, const uint8_t **restored_out);
void rs_decoder_free(rs_decoder *dec);

/* -------------------------------------------- batched device entry points
 * Device-resident, asynchronous on `stream`, thread-safe, stateless apart
 * from a per-(k, m, flags[, erasure pattern]) plan cache. Stripes are
 * independent; shards of one stripe are contiguous (shard stride =
 * shard_bytes); a stripe stride of 0 means packed.
 *   d_original: [n_stripes][k][shard_bytes]  (stride original_stripe_stride)
 *   d_recovery: [n_stripes][m][shard_bytes]  (stride recovery_stripe_stride) */
int rs_encode_batch_dev(uint64_t original_count, uint64_t recovery_count, size_t shard_bytes, uint64_t n_stripes,
                        const void *d_original, uint64_t original_stripe_stride, void *d_recovery,
                        uint64_t recovery_stripe_stride, uint32_t flags, rs_stream_t stream);

/* Reconstruct the missing originals of every stripe; one erasure pattern for
 * the whole batch. present: host array of k+m flags (originals, then
 * recovery). Missing slots of d_original/d_recovery are never read.
 *   d_restored: [n_stripes][e][shard_bytes], e = missing originals, ascending index. */
int rs_reconstruct_batch_dev(uint64_t original_count, uint64_t recovery_count, size_t shard_bytes,
                             uint64_t n_stripes, const uint8_t *present, const void *d_original,
                             uint64_t original_stripe_stride, const void *d_recovery,
                             uint64_t recovery_stripe_stride, void *d_restored, uint64_t restored_stripe_stride,
                             uint32_t flags, rs_stream_t stream);

/* Reconstruct with a per-stripe erasure pattern (§8f rank 2). d_present: DEVICE
 * array, n_stripes rows of k+m flags (row stride present_stride, 0 = k+m). The
 * erasure locator (Generic.zig:200-215, two 64K-point FWHTs) is evaluated per
 * stripe on the GPU. Stripe s restores its missing originals, ascending, into
 * slots [0, e_s) of its d_restored row ([n][max_e][shard_bytes]); slots >= e_s
 * are not written. d_status (device, n int32, may be NULL) receives per stripe
 * RS_OK, RS_ERR_NOT_ENOUGH_SHARDS (< k present) or RS_ERR_INVALID_ARGUMENT
 * (e_s > max_e: restored slots past max_e are dropped). */
int rs_reconstruct_batch_dev_patterns(uint64_t original_count, uint64_t recovery_count, size_t shard_bytes,
                                      uint64_t n_stripes, const uint8_t *d_present, uint64_t present_stride,
                                      uint32_t max_e, const void *d_original, uint64_t original_stripe_stride,
                                      const void *d_recovery, uint64_t recovery_stripe_stride, void *d_restored,
                                      uint64_t restored_stripe_stride, int32_t *d_status, uint32_t flags,
                                      rs_stream_t stream);

/* -------------------------------------- host-resident batches (end to end)
 * Same layouts and semantics as the *_dev calls, but the batch lives in HOST
 * memory: the library streams it through HBM in slices on a 2-slot (RS_AMD_HOST_SLOTS)
 * H2D -> kernel -> D2H pipeline on its own streams (PCIe full duplex overlapped
 * with compute) and returns when the results are in host memory. Pinned host
 * buffers (hipHostMalloc / hipHostRegister / torch pin_memory) run at PCIe rate;
 * pageable buffers are copied by host threads (up to 16, RS_AMD_HOST_THREADS) through the
 * ring's own pinned staging (RS_AMD_HOST_STAGE=0: the HIP runtime's pageable path instead).
 * A reconstruct reads only the present shards: one copy per run of consecutive present
 * rows (RS_AMD_HOST_GAP=n also copies gaps of up to n missing rows, bytes never read),
 * in slices of 256 MiB (RS_AMD_HOST_SLICE_MB) widened up to 1 GiB while the narrowest
 * run's copy would move less than 8 MiB. Ring copies use the 2D copy form (faster than the
 * 1D one from pinned memory; RS_AMD_HOST_COPY2D=0 reverts). The ring's device buffers persist
 * per device. */
int rs_encode_batch_host(uint64_t original_count, uint64_t recovery_count, size_t shard_bytes, uint64_t n_stripes,
                         const void *h_original, uint64_t original_stripe_stride, void *h_recovery,
                         uint64_t recovery_stripe_stride, uint32_t flags);
int rs_reconstruct_batch_host(uint64_t original_count, uint64_t recovery_count, size_t shard_bytes,
                              uint64_t n_stripes, const uint8_t *present, const void *h_original,
                              uint64_t original_stripe_stride, const void *h_recovery,
                              uint64_t recovery_stripe_stride, void *h_restored, uint64_t restored_stripe_stride,
                              uint32_t flags);

/* The same host-memory batches split over several GPUs of the node: device i of
 * devices[0..n_devices) (NULL = every visible device) takes the contiguous stripe
 * range [i*n/D, (i+1)*n/D) and runs it on its own worker thread and staging ring
 * (stripes are independent: no exchange between devices). Returns the first
 * failing device's status (its message in rs_last_error) after every worker ended. */
int rs_encode_batch_host_multi(uint64_t original_count, uint64_t recovery_count, size_t shard_bytes,
                               uint64_t n_stripes, const void *h_original, uint64_t original_stripe_stride,
                               void *h_recovery, uint64_t recovery_stripe_stride, uint32_t flags,
                               const int *devices, int n_devices);
int rs_reconstruct_batch_host_multi(uint64_t original_count, uint64_t recovery_count, size_t shard_bytes,
                                    uint64_t n_stripes, const uint8_t *present, const void *h_original,
                                    uint64_t original_stripe_stride, const void *h_recovery,
                                    uint64_t recovery_stripe_stride, void *h_restored,
                                    uint64_t restored_stripe_stride, uint32_t flags, const int *devices,
                                    int n_devices);

/* Which device kernel a call would run on in its steady state ("net_encode_i10_o4",
 * "encode_reg_w4_nv4", "decode_matrix_e4_nv4", "encode_generic_nv1",
 * "net_fft_encode_i200_o55", "net_fft_pdecode_i200_o55", ...), assuming 16-byte aligned
 * buffers. present: k+m flags as for rs_reconstruct_batch_dev, or NULL for "the first
 * min(k, m) originals lost". net_<role>_* = bit-sliced XOR network (or bit-sliced FFT
 * kernel, net_fft_*) generated for the plan and compiled with hipRTC on first use (shards of
 * 1 / 2 KiB or whole 4 KiB units, <= 64 outputs; up to 64 input blocks compile in the call,
 * larger maps in the background; disable with RS_AMD_JIT=0). A prediction: the kernels a
 * call actually launched are in rs_last_kernels. */
const char *rs_encode_kernel_name(uint64_t original_count, uint64_t recovery_count, size_t shard_bytes);
const char *rs_reconstruct_kernel_name(uint64_t original_count, uint64_t recovery_count, size_t shard_bytes,
                                       const uint8_t *present);
/* Path rs_reconstruct_batch_dev_patterns takes for these arguments (16-byte aligned
 * buffers): "psyn_k<k>_m<m>" (k <= 256, m <= 8, whole 4 KiB units: the code's syndrome
 * network + a per-stripe solve), "fft_decode" (chunk 16 / 32 / 64 codes with max_e >= 0.6 m,
 * or shards of whole 2 KiB units: the fused FFT reconstruct with per-stripe decode blocks
 * built on the GPU), "fft_syndromes+psyn_solve" (chunk 16 / 32 / 64 otherwise: FFT syndromes
 * with per-stripe masks + the e x e solve in output groups of 8), "pattern_matrix"
 * (per-stripe e x k table matrices, W <= 32, max_e <= 8) or "pattern_fft" (the reference's
 * decode on the generic FFT kernels: D1, D2-dropping codes, everything else) or
 * "pattern_fft_low" (low-rate codes: the same decode in the low-rate layout). These are
 * what a call is planned to run; rs_last_kernels reports what it did run. */
const char *rs_patterns_kernel_name(uint64_t original_count, uint64_t recovery_count, size_t shard_bytes,
                                    uint32_t max_e, uint32_t flags);

/* Per-pattern kernels of wide codes compile in a background thread. A wide-code pattern's
 * first calls run the fused FFT reconstruct with the pattern as data (rs_fft_decode_*,
 * nothing compiled per pattern). One steady-state kernel per pattern is then built on the
 * background worker, behind the full plan's build: a network where one beats the fused
 * kernel (few losses: the direct map, queued at the pattern's second call; RS_AMD_FDEC=0:
 * the e x e syndrome map), else the fused kernel with the pattern compiled in
 * (rs_fft_pdecode_*, k <= 256; RS(200,55): 8-16 s of hipRTC), queued at the pattern's
 * RS_AMD_PDEC_AFTER-th call (default 2). The pattern-compiled kernels are bounded: at most
 * RS_AMD_PDEC_MAX (default 32) patterns per code and device (later patterns keep the
 * pattern-as-data kernel), and none is queued while more than RS_AMD_PDEC_QUEUE (default 2)
 * jobs wait on the worker (a later call retries). The calls run the first form until the
 * steady-state kernel is loaded. rs_net_wait blocks until the worker is idle (no plan build
 * or compile queued or running): after two calls + rs_net_wait the next call runs the
 * pattern's steady-state kernel (rs_reconstruct_warm gets there at once). RS_AMD_JIT_SYNC=1
 * compiles in the calling thread instead. Returns RS_OK. */
int rs_net_wait(void);

/* Drive one erasure pattern of rs_reconstruct_batch_dev (same arguments) to its steady
 * state without running a batch: build its full plan and compile and load every kernel
 * its calls will launch, blocking until done. The next call runs the steady-state kernel
 * (check with rs_last_kernels). */
int rs_reconstruct_warm(uint64_t original_count, uint64_t recovery_count, size_t shard_bytes, const uint8_t *present,
                        uint32_t flags);

/* The kernels the calling thread's most recent compute call (the *_dev, *_host, one-shot,
 * Encoder/Decoder and engine entry points) launched, in launch order, ';'-separated,
 * consecutive repeats collapsed: hipRTC kernels by symbol (rs_net_encode_i10_o4_<hash>,
 * rs_fft_decode_k200_m55_..., the names rocprofv3 reports), precompiled ones by their
 * rs_*_kernel_name form (encode_reg_w4_nv4, k_erasure_logs, ...). Host batches launch on
 * worker threads and are recorded there, not here. Valid until the thread's next call. */
const char *rs_last_kernels(void);

/* ------------------------------------------------ fault injection (tests only)
 * The reference runs its encode under std.testing.checkAllAllocationFailures
 * (tests.zig:131-156): every allocation of the call fails in turn and must surface as
 * error.OutOfMemory with nothing leaked. Here every allocation the library makes — plan
 * objects, device and stream-ordered buffers, pinned staging — is counted; after
 * rs_debug_fail_alloc(n) the n-th one (from 0, all threads) fails as if out of memory and
 * the call returns RS_ERR_OUT_OF_MEMORY. n < 0 disarms. Returns the number of allocations
 * counted since the previous rs_debug_fail_alloc call. */
int64_t rs_debug_fail_alloc(int64_t n);
/* Drop every cache holding device or pinned memory (plans, device tables, staging rings,
 * pooled one-shot contexts; compiled kernels stay loaded), after any background plan build
 * finished. *pooled_contexts (optional) = one-shot contexts left in the pool (0). */
int rs_debug_release_caches(uint64_t *pooled_contexts);
/* Host erasure locators (root.zig:277-289, Generic.zig:200-215 evalPoly): the library sums a
 * small erased set's log terms point by point instead of the two 65536-point transforms.
 * Evaluates both for `received` (high rate: recovery at [0, m), originals at [C, C + k),
 * C = ceilPow2(m); low != 0: rs_gf.hpp erasure_logs_low's layout) and returns the number of
 * positions below ceilPow2(C + k) (low: ceilPow2(C + m)) where they differ mod 65535; -1 on
 * invalid arguments. Host only, no device. */
int64_t rs_debug_erasure_logs_check(uint64_t k, uint64_t m, const uint8_t *received, int low);
/* Measurement builds of the FFT kernels (RS_AMD_FFT_DEBUG bit 6, rs_fftnet.cpp): every wave
 * of workgroup 0 stamps s_memtime around each barrier of its third unit; copies the current
 * device's 8 x 64 stamps (wave-major) to out[0, min(n, 512)). */
int rs_debug_fft_stamps(uint64_t *out, uint64_t n);

/* hipRTC activity of this process: kernels compiled, code objects found in the on-disk
 * cache ($RS_AMD_CACHE_DIR, else $XDG_CACHE_HOME/rs_amd or ~/.cache/rs_amd; empty = off),
 * modules loaded. Any pointer may be NULL. */
int rs_jit_stats(uint64_t *compiles, uint64_t *cache_hits, uint64_t *modules);

/* Plan-time network kernel: generate the bit-sliced network of an encode (present
 * == NULL) or of one reconstruct pattern and compile it with hipRTC for gfx950, without
 * loading it (no device needed: a build check). *compile_ms (optional) = compile time.
 * RS_ERR_INVALID_ARGUMENT if the shape has no network form, RS_ERR_DEVICE if hipRTC fails. */
int rs_net_compile_check(uint64_t original_count, uint64_t recovery_count, const uint8_t *present,
                         uint32_t flags, double *compile_ms);

/* Generate the per-stripe syndrome-network reconstruct kernels of
 * rs_reconstruct_batch_dev_patterns (rs_psyn.hpp) and compile them with hipRTC (no
 * device): for k <= 256, m <= 8 the code's fixed k -> m syndrome network plus the
 * per-stripe e x e solve; for chunk 16 / 32 / 64 codes the FFT syndrome kernel with
 * per-stripe masks plus the generic solve. RS_ERR_INVALID_ARGUMENT if the code has none. */
int rs_psyn_compile_check(uint64_t original_count, uint64_t recovery_count, uint32_t flags, double *compile_ms,
                          uint64_t *code_bytes);
/* Bit-sliced FFT encode kernel (wide codes, chunk 32 / 64): generate
 * it for (original_count, recovery_count, flags) and compile it with hipRTC, without
 * loading it (a build check; no device needed). Optional outputs: compile time, code
 * object bytes, and the generated kernel's VALU instruction estimate per 2 KiB unit
 * (all waves). RS_ERR_INVALID_ARGUMENT if the code has no such kernel. */
int rs_fft_compile_check(uint64_t original_count, uint64_t recovery_count, uint32_t flags, double *compile_ms,
                         uint64_t *code_bytes, uint64_t *valu_ops);
/* Host check of that kernel's arithmetic (its butterfly schedule with its (u, v)
 * coordinate matrices on scalar symbols, against the codec's scalar encode, with
 * the data shards flagged in skip (k bytes, NULL = none) read as zero): *mismatches
 * = wrong parity symbols over `trials` random stripes. */
int rs_fft_selftest(uint64_t original_count, uint64_t recovery_count, uint32_t flags, const uint8_t *skip,
                    int trials, uint64_t *mismatches);

/* Fused FFT reconstruct of wide codes (replaces the reference's
 * Decoder.decode, root.zig:268-335, for chunk 16 / 32 / 64 codes, corrected multiply):
 * the syndromes of e recovery rows and the erasure-locator decode in one kernel, the
 * pattern as data. rs_fft_decode_compile_check generates and compiles it (no device);
 * rs_fft_decode_selftest runs its schedule on scalar symbols (host) for `trials` random
 * stripes losing e originals (and random surplus recovery shards) against the data:
 * *mismatches = wrong restored symbols. RS_ERR_INVALID_ARGUMENT if the code has no such
 * kernel or e > recovery_count. */
int rs_fft_decode_compile_check(uint64_t original_count, uint64_t recovery_count, double *compile_ms,
                                uint64_t *code_bytes);
/* The same kernel with one erasure pattern compiled in (present: k + m flags): the locator
 * scalars as constant multiplies, rows, blocks and outputs static (the steady state of a
 * pattern reused across batches). RS_ERR_NOT_ENOUGH_SHARDS if the pattern cannot decode. */
int rs_fft_pdecode_compile_check(uint64_t original_count, uint64_t recovery_count, const uint8_t *present,
                                 double *compile_ms, uint64_t *code_bytes);
int rs_fft_decode_selftest(uint64_t original_count, uint64_t recovery_count, uint32_t erased, int trials,
                           uint64_t *mismatches);

/* Host check of the low-rate reconstruct's algebra (no device): `trials` random stripes
 * of one symbol per shard, encoded by the low-rate encode, lose 1..min(k, m) random
 * originals plus random recovery shards (>= k present), and are restored by the
 * erasure-locator decode in the low-rate layout (rs_lowrate.cpp). *mismatches = wrong
 * restored symbols. RS_ERR_INVALID_ARGUMENT for a high-rate code. */
int rs_lowrate_selftest(uint64_t original_count, uint64_t recovery_count, int trials, uint64_t seed,
                        uint64_t *mismatches);

/* ---------------------------------------- Engine seam (Generic.zig), test shim
 * The reference's comptime Engine interface (root.zig:10-12) at per-call
 * granularity, run on the GPU over a HOST buffer of shard_count shards of
 * shard_bytes (copied in and out). For stage-by-stage parity only. */
int rs_engine_fft(uint8_t *shards, uint64_t shard_count, size_t shard_bytes, uint64_t pos, uint64_t size,
                  uint64_t truncated_size, uint64_t skew_delta, uint32_t flags);  /* Generic.zig:15 */
int rs_engine_ifft(uint8_t *shards, uint64_t shard_count, size_t shard_bytes, uint64_t pos, uint64_t size,
                   uint64_t truncated_size, uint64_t skew_delta, uint32_t flags); /* Generic.zig:80 */
int rs_engine_mul_scalar(uint8_t *chunks, size_t bytes, uint16_t log_m, uint32_t flags); /* Generic.zig:220 */
/* Generic.zig:200 evalPoly over 65536 u16 erasure flags, in place (host FWHT). */
int rs_engine_eval_poly(uint16_t *erasures, uint64_t truncated_size);

/* ---------------------------------------------------- tables (tables.zig) */
const uint16_t *rs_table_exp(void);       /* [65536] */
const uint16_t *rs_table_log(void);       /* [65536] */
const uint16_t *rs_table_skew(void);      /* [65535] */
const uint16_t *rs_table_log_walsh(void); /* [65536] */
/* tables.zig:94-118 `mul_128: [65536]Lut`, `Lut = [2][4]u128`: for multiplier log_m, byte
 * [log_m][h][i][j] = byte h (0 low, 1 high) of mul16(j << 4i, log_m) — the x86 engine's
 * pshufb nibble tables (8 MiB, built on the first call; the GPU kernels use their own
 * v_perm / bit-sliced forms). NULL if it cannot be allocated. */
const uint8_t *rs_table_mul_128(void);

#ifdef __cplusplus
}
#endif
#endif /* REEDSOL_AMD_H */
