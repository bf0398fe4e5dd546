/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the usebeforefree/reed-solomon-cc (Zig, snapshot
 * 2025-12-12) high-rate Reed-Solomon codec: GF(2^16) in a Cantor basis,
 * Lin-Chung-Han additive FFT, Leopard-style encode/decode.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load or call this library, and only as the checker / the CPU baseline.
 * The product path (reed-solomon-cc_amd/) never links or calls it.
 *
 * Parity is pinned by the reference's own golden vectors
 * (src/tests/encode_data.zon, Generic.zig:317-455 KATs, tests.zig:61-102
 * exhaustive roundtrip); see tests/test_oracle_golden.py.
 *
 * Quirk switch:
 *   RSO_CORRECTED   — default, roundtrip-correct arithmetic and schedule;
 *   RSO_Q_D1        — Generic.zig:283 uses t1_hi for nibble 0 of the hi product;
 *   RSO_Q_D2        — root.zig:151 drops the last full chunk when k%chunk==0.
 * D3..D6 (L>1 slice-length bugs) are NOT reproduced: they crash the literal
 * reference; the oracle is L-generic (SURVEY.md §A.6 column independence).
 */
#ifndef RS_ORACLE_H
#define RS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  RSO_CORRECTED = 0,
  RSO_Q_D1 = 1,
  RSO_Q_D2 = 2,
  RSO_REF_LITERAL = RSO_Q_D1 | RSO_Q_D2,
};

/* error codes — same numbering as include/reedsol.h (mirrors root.zig errors) */
enum {
  RSO_OK = 0,
  RSO_ERR_TOO_FEW_ORIGINAL_SHARDS = 1,
  RSO_ERR_NOT_ENOUGH_SHARDS = 2,
  RSO_ERR_INVALID_SHARD_SIZE = 3,
  RSO_ERR_UNSUPPORTED_SHARD_COUNT = 4,
  RSO_ERR_TOO_MANY_ORIGINAL_SHARDS = 5,
  RSO_ERR_DIFFERENT_SHARD_SIZE = 6,
  RSO_ERR_INVALID_SHARD_INDEX = 7,
  RSO_ERR_DUPLICATE_SHARD_INDEX = 8,
  RSO_ERR_TOO_MANY_SHARDS = 9,
  RSO_ERR_OUT_OF_MEMORY = 10,
  RSO_ERR_LOW_RATE_UNSUPPORTED = 12,
  RSO_ERR_SHARD_TAIL_UNSUPPORTED = 13, /* no longer returned: tails use the layout of root.zig:338-348 */
};

void rso_init(void);

/* tables (tables.zig) */
const uint16_t *rso_exp(void);       /* [65536] */
const uint16_t *rso_log(void);       /* [65536] */
const uint16_t *rso_skew(void);      /* [65535] */
const uint16_t *rso_log_walsh(void); /* [65536] */
const uint8_t *rso_mul128(void);     /* [65536][2][4][16] */

uint16_t rso_mul16(uint16_t x, uint16_t log_m);
uint16_t rso_add_mod(uint32_t x, uint32_t y);
uint16_t rso_sub_mod(uint32_t x, uint32_t y);

/* engine (Generic.zig) — `data` is a [shard_count][L][64] buffer */
void rso_mul_chunk(const uint8_t *in, uint8_t *out, uint16_t log_m, int quirks);
void rso_fft(uint8_t *data, size_t L, uint64_t pos, uint64_t size, uint64_t trunc, uint64_t skew_delta,
             int quirks);
void rso_ifft(uint8_t *data, size_t L, uint64_t pos, uint64_t size, uint64_t trunc, uint64_t skew_delta,
              int quirks);
void rso_fft_partial(uint8_t *x, uint8_t *y, size_t nchunks, uint16_t log_m, int quirks);
void rso_ifft_partial(uint8_t *x, uint8_t *y, size_t nchunks, uint16_t log_m, int quirks);
void rso_mul_scalar(uint8_t *chunks, size_t nchunks, uint16_t log_m, int quirks);
void rso_fwht(uint16_t *data, uint64_t m);
void rso_eval_poly(uint16_t *erasures, uint64_t trunc);

/* rate selection (root.zig:397-415): 1 = high rate, 0 = low rate, <0 = -error */
int rso_use_high_rate(uint64_t k, uint64_t m);

/* codec (root.zig) — caller owns every buffer; any even shard_bytes (a tail of
 * shard_bytes % 64 bytes uses the last-chunk layout root.zig:338-348 implies) */
int rso_encode(uint64_t k, uint64_t m, size_t shard_bytes, const uint8_t *const *original,
               uint8_t *const *recovery_out, int quirks);
/* low-rate encode (absent from the reference, parity unpinned; see rs_oracle.c) */
int rso_encode_low(uint64_t k, uint64_t m, size_t shard_bytes, const uint8_t *const *original,
                   uint8_t *const *recovery_out, int quirks);
/* original[i] / recovery[i] == NULL marks a missing shard; restored_out has k
 * slots and receives every original (copied for present ones). */
int rso_decode(uint64_t k, uint64_t m, size_t shard_bytes, const uint8_t *const *original,
               const uint8_t *const *recovery, uint8_t *const *restored_out, int quirks);

/* batched, stripe-parallel on `threads` host threads.
 * data:   [n_stripes][k][shard_bytes]
 * parity: [n_stripes][m][shard_bytes]                                   */
int rso_encode_batch(uint64_t k, uint64_t m, size_t shard_bytes, size_t n_stripes, const uint8_t *data,
                     uint8_t *parity, int quirks, int threads);
/* present: k+m flags (originals then recovery), shared by every stripe.
 * shards: [n_stripes][k+m][shard_bytes] (missing slots are not read)
 * restored: [n_stripes][e][shard_bytes], e = number of missing originals, ascending */
int rso_reconstruct_batch(uint64_t k, uint64_t m, size_t shard_bytes, size_t n_stripes, const uint8_t *present,
                          const uint8_t *shards, uint8_t *restored, int quirks, int threads);

int rso_have_avx2(void);
void rso_force_scalar(int on);

/* benchmarks.zig protocol (mean ns per insert + encode), natively timed */
double rso_bench_encode(uint64_t k, uint64_t m, size_t shard_bytes, uint64_t iters, int quirks);

#ifdef __cplusplus
}
#endif
#endif
