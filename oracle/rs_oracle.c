/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see rs_oracle.h).
 *
 * Plain-C restatement of usebeforefree/reed-solomon-cc. Every function cites
 * the reference file:line it restates (paths relative to the reference repo).
 * The shard buffer generalises the reference's `Shards` ([count*L][64]u8,
 * root.zig:350-395) to any L = shard_bytes/64 with the slice lengths the
 * code intends (× L), which is what column independence
 * requires; at L == 1 it is the literal reference.
 *
 * Two multiply back ends, bit-identical: portable scalar (the reference's
 * `shuffle` fallback, Generic.zig:305-313) and AVX2 vpshufb (the reference's
 * x86-64 LLVM path, Generic.zig:300-303), selected at run time. The AVX2 one
 * is what the CPU baseline times.
 */
#define _GNU_SOURCE
#include "rs_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#if defined(__x86_64__)
#include <immintrin.h>
#define RSO_X86 1
#else
#define RSO_X86 0
#endif

/* ---------------------------------------------------------------- gf.zig:3-13 */
#define GF_ORDER 65536u
#define GF_MODULUS 65535u
#define GF_POLY 65581u
static const uint16_t CANTOR[16] = {0x0001, 0xACCA, 0x3C0E, 0x163E, 0xC582, 0xED2E, 0x914C, 0x4012,
                                    0x6C98, 0x10D8, 0x6A72, 0xB900, 0xFDB8, 0xFB34, 0xFF38, 0x991E};

static uint16_t g_exp[GF_ORDER];
static uint16_t g_log[GF_ORDER];
static uint16_t g_skew[GF_MODULUS];
static uint16_t g_log_walsh[GF_ORDER];
static uint8_t (*g_mul128)[2][4][16]; /* [65536][2][4][16] = 8 MiB */
static int g_inited = 0;
static int g_force_scalar = 0;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

/* ------------------------------------------------------------ utilities.zig */
/* utilities.zig:10-13 */
uint16_t rso_add_mod(uint32_t x, uint32_t y) {
  uint32_t sum = x + y;
  return (uint16_t)(sum + (sum >> 16));
}
/* utilities.zig:15-18 */
uint16_t rso_sub_mod(uint32_t x, uint32_t y) {
  uint32_t dif = x + GF_MODULUS - y;
  return (uint16_t)(dif + (dif >> 16));
}
/* utilities.zig:5-8 */
static uint16_t mul16_t(uint16_t x, uint16_t log_m, const uint16_t *exp, const uint16_t *log) {
  if (x == 0) return 0;
  return exp[rso_add_mod(log[x], log_m)];
}

/* ------------------------------------------------------ walsh_hadamard.zig */
/* walsh_hadamard.zig:58-62 (fwht2) + 38-55 (fwht4) */
static void fwht4(uint16_t *d, uint64_t off, uint64_t stride) {
  uint64_t x0 = off, x1 = off + stride, x2 = off + 2 * stride, x3 = off + 3 * stride;
  uint16_t s0 = rso_add_mod(d[x0], d[x1]), d0 = rso_sub_mod(d[x0], d[x1]);
  uint16_t s1 = rso_add_mod(d[x2], d[x3]), d1 = rso_sub_mod(d[x2], d[x3]);
  uint16_t s2 = rso_add_mod(s0, s1), d2 = rso_sub_mod(s0, s1);
  uint16_t s3 = rso_add_mod(d0, d1), d3 = rso_sub_mod(d0, d1);
  d[x0] = s2;
  d[x1] = s3;
  d[x2] = d2;
  d[x3] = d3;
}
/* walsh_hadamard.zig:16-31 */
void rso_fwht(uint16_t *data, uint64_t m) {
  uint64_t dist = 1, stride = 4;
  while (stride <= GF_ORDER) {
    for (uint64_t r = 0; r < m; r += stride)
      for (uint64_t off = r; off < r + dist; off++) fwht4(data, (uint16_t)off, (uint16_t)dist);
    dist = stride;
    stride *= 4;
  }
}

/* ---------------------------------------------------------------- tables.zig */
static void build_tables(void) {
  static uint16_t exp[GF_ORDER], log[GF_ORDER];
  /* tables.zig:22-31: LFSR; note `exp` first holds logs */
  uint64_t state = 1;
  memset(exp, 0, sizeof exp);
  memset(log, 0, sizeof log);
  for (uint32_t i = 0; i < GF_MODULUS; i++) {
    exp[state] = (uint16_t)i;
    state <<= 1;
    if (state >= GF_ORDER) state ^= GF_POLY;
  }
  exp[0] = GF_MODULUS;
  /* tables.zig:35-41: Cantor basis */
  log[0] = 0;
  for (int i = 0; i < 16; i++) {
    uint32_t width = 1u << i;
    for (uint32_t j = 0; j < width; j++) log[j + width] = log[j] ^ CANTOR[i];
  }
  /* tables.zig:43-45 */
  for (uint32_t i = 0; i < GF_ORDER; i++) log[i] = exp[log[i]];
  for (uint32_t i = 0; i < GF_ORDER; i++) exp[log[i]] = (uint16_t)i;
  exp[GF_MODULUS] = exp[0];
  memcpy(g_exp, exp, sizeof exp);
  memcpy(g_log, log, sizeof log);

  /* tables.zig:60-87: LCH skew factors */
  static uint16_t skew[GF_MODULUS];
  uint16_t temp[15];
  memset(skew, 0, sizeof skew);
  for (int i = 1; i < 16; i++) temp[i - 1] = (uint16_t)(1u << i);
  for (int m = 0; m < 15; m++) {
    uint64_t step = 1ull << (m + 1);
    uint16_t backwards = (uint16_t)((1u << m) - 1);
    skew[backwards] = 0;
    for (int i = m; i < 15; i++) {
      uint32_t s = 1u << (i + 1);
      for (uint32_t j = backwards; j < s; j += (uint32_t)step) skew[j + s] = skew[j] ^ temp[i];
    }
    temp[m] = (uint16_t)(GF_MODULUS - log[mul16_t(temp[m], log[temp[m] ^ 1], exp, log)]);
    for (int i = m + 1; i < 15; i++) {
      uint16_t sum = rso_add_mod(log[temp[i] ^ 1], temp[m]);
      temp[i] = mul16_t(temp[i], sum, exp, log);
    }
  }
  for (uint32_t i = 0; i < GF_MODULUS; i++) skew[i] = log[skew[i]];
  memcpy(g_skew, skew, sizeof skew);

  /* tables.zig:99-118: per-multiplier nibble LUTs */
  g_mul128 = malloc((size_t)GF_ORDER * sizeof *g_mul128);
  for (uint32_t lm = 0; lm < GF_ORDER; lm++)
    for (int i = 0; i < 4; i++)
      for (uint32_t j = 0; j < 16; j++) {
        uint16_t p = mul16_t((uint16_t)(j << (4 * i)), (uint16_t)lm, exp, log);
        g_mul128[lm][0][i][j] = (uint8_t)p;
        g_mul128[lm][1][i][j] = (uint8_t)(p >> 8);
      }

  /* tables.zig:146-147 */
  memcpy(g_log_walsh, log, sizeof log);
  rso_fwht(g_log_walsh, GF_ORDER);
  g_inited = 1;
}

void rso_init(void) { pthread_once(&g_once, build_tables); }
const uint16_t *rso_exp(void) { rso_init(); return g_exp; }
const uint16_t *rso_log(void) { rso_init(); return g_log; }
const uint16_t *rso_skew(void) { rso_init(); return g_skew; }
const uint16_t *rso_log_walsh(void) { rso_init(); return g_log_walsh; }
const uint8_t *rso_mul128(void) { rso_init(); return (const uint8_t *)g_mul128; }
uint16_t rso_mul16(uint16_t x, uint16_t log_m) { rso_init(); return mul16_t(x, log_m, g_exp, g_log); }

/* ------------------------------------------------------------ Generic.zig */
int rso_have_avx2(void) {
#if RSO_X86
  return __builtin_cpu_supports("avx2") && __builtin_cpu_supports("ssse3");
#else
  return 0;
#endif
}
void rso_force_scalar(int on) { g_force_scalar = on; }
static int use_avx2(void) { return !g_force_scalar && rso_have_avx2(); }

/* Generic.zig:275-298 `mul` + portable `shuffle` (305-313), one 64-B chunk:
 * bytes [0,32) are the lo bytes and [32,64) the hi bytes of 32 symbols. */
static inline void mul_chunk_scalar(const uint8_t *in, uint8_t *prod, uint16_t log_m, int quirks) {
  const uint8_t(*t)[4][16] = g_mul128[log_m];
  const uint8_t *hi0 = (quirks & RSO_Q_D1) ? t[1][1] : t[1][0]; /* D1: Generic.zig:283 */
  for (int j = 0; j < 32; j++) {
    uint8_t lo = in[j], hi = in[32 + j];
    uint8_t n0 = lo & 15, n1 = lo >> 4, n2 = hi & 15, n3 = hi >> 4;
    prod[j] = t[0][0][n0] ^ t[0][1][n1] ^ t[0][2][n2] ^ t[0][3][n3];
    prod[32 + j] = hi0[n0] ^ t[1][1][n1] ^ t[1][2][n2] ^ t[1][3][n3];
  }
}

#if RSO_X86
typedef struct {
  __m256i t0l, t1l, t2l, t3l, t0h, t1h, t2h, t3h;
} lut_avx2;

/* Generic.zig:252-273 Lut.init + broadcast */
__attribute__((target("avx2"))) static inline lut_avx2 lut_init_avx2(uint16_t log_m, int quirks) {
  const uint8_t(*t)[4][16] = g_mul128[log_m];
  lut_avx2 L;
  L.t0l = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t[0][0]));
  L.t1l = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t[0][1]));
  L.t2l = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t[0][2]));
  L.t3l = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t[0][3]));
  L.t0h = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t[1][(quirks & RSO_Q_D1) ? 1 : 0]));
  L.t1h = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t[1][1]));
  L.t2h = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t[1][2]));
  L.t3h = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i *)t[1][3]));
  return L;
}

/* Generic.zig:275-298 with vpshufb (Generic.zig:300-303) */
__attribute__((target("avx2"))) static inline void mul_avx2(__m256i lo, __m256i hi, const lut_avx2 *L,
                                                            __m256i *plo, __m256i *phi) {
  const __m256i nib = _mm256_set1_epi8(0x0f);
  __m256i d0 = _mm256_and_si256(lo, nib);
  __m256i d1 = _mm256_and_si256(_mm256_srli_epi64(lo, 4), nib);
  __m256i d2 = _mm256_and_si256(hi, nib);
  __m256i d3 = _mm256_and_si256(_mm256_srli_epi64(hi, 4), nib);
  __m256i pl = _mm256_shuffle_epi8(L->t0l, d0);
  __m256i ph = _mm256_shuffle_epi8(L->t0h, d0);
  pl = _mm256_xor_si256(pl, _mm256_shuffle_epi8(L->t1l, d1));
  ph = _mm256_xor_si256(ph, _mm256_shuffle_epi8(L->t1h, d1));
  pl = _mm256_xor_si256(pl, _mm256_shuffle_epi8(L->t2l, d2));
  ph = _mm256_xor_si256(ph, _mm256_shuffle_epi8(L->t2h, d2));
  pl = _mm256_xor_si256(pl, _mm256_shuffle_epi8(L->t3l, d3));
  ph = _mm256_xor_si256(ph, _mm256_shuffle_epi8(L->t3h, d3));
  *plo = pl;
  *phi = ph;
}

/* Generic.zig:149-169 */
__attribute__((target("avx2"))) static void fft_partial_avx2(uint8_t *x, uint8_t *y, size_t n, uint16_t lm,
                                                             int quirks) {
  lut_avx2 L = lut_init_avx2(lm, quirks);
  for (size_t c = 0; c < n; c++, x += 64, y += 64) {
    __m256i xl = _mm256_loadu_si256((const __m256i *)x), xh = _mm256_loadu_si256((const __m256i *)(x + 32));
    __m256i yl = _mm256_loadu_si256((const __m256i *)y), yh = _mm256_loadu_si256((const __m256i *)(y + 32));
    __m256i pl, ph;
    mul_avx2(yl, yh, &L, &pl, &ph);
    xl = _mm256_xor_si256(xl, pl);
    xh = _mm256_xor_si256(xh, ph);
    _mm256_storeu_si256((__m256i *)x, xl);
    _mm256_storeu_si256((__m256i *)(x + 32), xh);
    _mm256_storeu_si256((__m256i *)y, _mm256_xor_si256(yl, xl));
    _mm256_storeu_si256((__m256i *)(y + 32), _mm256_xor_si256(yh, xh));
  }
}

/* Generic.zig:171-192 */
__attribute__((target("avx2"))) static void ifft_partial_avx2(uint8_t *x, uint8_t *y, size_t n, uint16_t lm,
                                                              int quirks) {
  lut_avx2 L = lut_init_avx2(lm, quirks);
  for (size_t c = 0; c < n; c++, x += 64, y += 64) {
    __m256i xl = _mm256_loadu_si256((const __m256i *)x), xh = _mm256_loadu_si256((const __m256i *)(x + 32));
    __m256i yl = _mm256_loadu_si256((const __m256i *)y), yh = _mm256_loadu_si256((const __m256i *)(y + 32));
    yl = _mm256_xor_si256(yl, xl);
    yh = _mm256_xor_si256(yh, xh);
    _mm256_storeu_si256((__m256i *)y, yl);
    _mm256_storeu_si256((__m256i *)(y + 32), yh);
    __m256i pl, ph;
    mul_avx2(yl, yh, &L, &pl, &ph);
    _mm256_storeu_si256((__m256i *)x, _mm256_xor_si256(xl, pl));
    _mm256_storeu_si256((__m256i *)(x + 32), _mm256_xor_si256(xh, ph));
  }
}

/* Generic.zig:220-231 */
__attribute__((target("avx2"))) static void mul_scalar_avx2(uint8_t *x, size_t n, uint16_t lm, int quirks) {
  lut_avx2 L = lut_init_avx2(lm, quirks);
  for (size_t c = 0; c < n; c++, x += 64) {
    __m256i xl = _mm256_loadu_si256((const __m256i *)x), xh = _mm256_loadu_si256((const __m256i *)(x + 32));
    __m256i pl, ph;
    mul_avx2(xl, xh, &L, &pl, &ph);
    _mm256_storeu_si256((__m256i *)x, pl);
    _mm256_storeu_si256((__m256i *)(x + 32), ph);
  }
}

/* utilities.zig:20-27 */
__attribute__((target("avx2"))) static void xor_avx2(uint8_t *a, const uint8_t *b, size_t nchunks) {
  for (size_t c = 0; c < nchunks * 2; c++) {
    __m256i va = _mm256_loadu_si256((const __m256i *)(a + 32 * c));
    __m256i vb = _mm256_loadu_si256((const __m256i *)(b + 32 * c));
    _mm256_storeu_si256((__m256i *)(a + 32 * c), _mm256_xor_si256(va, vb));
  }
}
#endif

void rso_mul_chunk(const uint8_t *in, uint8_t *out, uint16_t log_m, int quirks) {
  rso_init();
  mul_chunk_scalar(in, out, log_m, quirks);
}

/* utilities.zig:20-27: a ^= b over 64-byte chunks */
static void xor_chunks(uint8_t *a, const uint8_t *b, size_t nchunks) {
#if RSO_X86
  if (use_avx2()) {
    xor_avx2(a, b, nchunks);
    return;
  }
#endif
  for (size_t i = 0; i < nchunks * 64; i++) a[i] ^= b[i];
}

/* Generic.zig:149-169: x ^= mul(y); y ^= x */
void rso_fft_partial(uint8_t *x, uint8_t *y, size_t n, uint16_t lm, int quirks) {
  rso_init();
#if RSO_X86
  if (use_avx2()) {
    fft_partial_avx2(x, y, n, lm, quirks);
    return;
  }
#endif
  uint8_t p[64];
  for (size_t c = 0; c < n; c++, x += 64, y += 64) {
    mul_chunk_scalar(y, p, lm, quirks);
    for (int i = 0; i < 64; i++) {
      x[i] ^= p[i];
      y[i] ^= x[i];
    }
  }
}

/* Generic.zig:171-192: y ^= x; x ^= mul(y) */
void rso_ifft_partial(uint8_t *x, uint8_t *y, size_t n, uint16_t lm, int quirks) {
  rso_init();
#if RSO_X86
  if (use_avx2()) {
    ifft_partial_avx2(x, y, n, lm, quirks);
    return;
  }
#endif
  uint8_t p[64];
  for (size_t c = 0; c < n; c++, x += 64, y += 64) {
    for (int i = 0; i < 64; i++) y[i] ^= x[i];
    mul_chunk_scalar(y, p, lm, quirks);
    for (int i = 0; i < 64; i++) x[i] ^= p[i];
  }
}

/* Generic.zig:220-231 */
void rso_mul_scalar(uint8_t *x, size_t n, uint16_t lm, int quirks) {
  rso_init();
#if RSO_X86
  if (use_avx2()) {
    mul_scalar_avx2(x, n, lm, quirks);
    return;
  }
#endif
  uint8_t p[64];
  for (size_t c = 0; c < n; c++, x += 64) {
    mul_chunk_scalar(x, p, lm, quirks);
    memcpy(x, p, 64);
  }
}

#define SHARD(data, L, s) ((data) + (size_t)(s) * (L) * 64)

/* Generic.zig:15-78 */
void rso_fft(uint8_t *data, size_t L, uint64_t pos, uint64_t size, uint64_t trunc, uint64_t skew_delta,
             int quirks) {
  rso_init();
  uint64_t distance = size >> 2, distance_4 = size;
  while (distance != 0) {
    for (uint64_t r = 0; r < trunc; r += distance_4) {
      uint64_t base = r + distance + skew_delta - 1;
      uint16_t m01 = g_skew[base], m02 = g_skew[base + distance], m23 = g_skew[base + 2 * distance];
      for (uint64_t i = r; i < r + distance; i++) {
        uint64_t p = pos + i;
        uint8_t *s0 = SHARD(data, L, p), *s1 = SHARD(data, L, p + distance);
        uint8_t *s2 = SHARD(data, L, p + 2 * distance), *s3 = SHARD(data, L, p + 3 * distance);
        if (m02 == GF_MODULUS) {
          xor_chunks(s2, s0, L);
          xor_chunks(s3, s1, L);
        } else {
          rso_fft_partial(s0, s2, L, m02, quirks);
          rso_fft_partial(s1, s3, L, m02, quirks);
        }
        if (m01 == GF_MODULUS) xor_chunks(s1, s0, L);
        else rso_fft_partial(s0, s1, L, m01, quirks);
        if (m23 == GF_MODULUS) xor_chunks(s3, s2, L);
        else rso_fft_partial(s2, s3, L, m23, quirks);
      }
    }
    distance_4 = distance;
    distance >>= 2;
  }
  if (distance_4 == 2) { /* Generic.zig:64-77 */
    for (uint64_t r = 0; r < trunc; r += 2) {
      uint16_t lm = g_skew[r + skew_delta];
      uint8_t *s0 = SHARD(data, L, pos + r), *s1 = SHARD(data, L, pos + r + 1);
      if (lm == GF_MODULUS) xor_chunks(s1, s0, L);
      else rso_fft_partial(s0, s1, L, lm, quirks);
    }
  }
}

/* Generic.zig:80-147 */
void rso_ifft(uint8_t *data, size_t L, uint64_t pos, uint64_t size, uint64_t trunc, uint64_t skew_delta,
              int quirks) {
  rso_init();
  uint64_t distance = 1, distance_4 = 4;
  while (distance_4 <= size) {
    for (uint64_t r = 0; r < trunc; r += distance_4) {
      uint64_t base = r + distance + skew_delta - 1;
      uint16_t m01 = g_skew[base], m02 = g_skew[base + distance], m23 = g_skew[base + 2 * distance];
      for (uint64_t i = r; i < r + distance; i++) {
        uint64_t p = pos + i;
        uint8_t *s0 = SHARD(data, L, p), *s1 = SHARD(data, L, p + distance);
        uint8_t *s2 = SHARD(data, L, p + 2 * distance), *s3 = SHARD(data, L, p + 3 * distance);
        if (m01 == GF_MODULUS) xor_chunks(s1, s0, L);
        else rso_ifft_partial(s0, s1, L, m01, quirks);
        if (m23 == GF_MODULUS) xor_chunks(s3, s2, L);
        else rso_ifft_partial(s2, s3, L, m23, quirks);
        if (m02 == GF_MODULUS) {
          xor_chunks(s2, s0, L);
          xor_chunks(s3, s1, L);
        } else {
          rso_ifft_partial(s0, s2, L, m02, quirks);
          rso_ifft_partial(s1, s3, L, m02, quirks);
        }
      }
    }
    distance = distance_4;
    distance_4 <<= 2;
  }
  if (distance < size) { /* Generic.zig:131-146 (slice lengths × L: D5 fixed) */
    uint16_t lm = g_skew[distance + skew_delta - 1];
    if (lm == GF_MODULUS) {
      xor_chunks(SHARD(data, L, pos + distance), SHARD(data, L, pos), distance * L);
    } else {
      for (uint64_t i = 0; i < distance; i++)
        rso_ifft_partial(SHARD(data, L, pos + i), SHARD(data, L, pos + distance + i), L, lm, quirks);
    }
  }
}

/* Generic.zig:200-215 */
void rso_eval_poly(uint16_t *erasures, uint64_t trunc) {
  rso_init();
  rso_fwht(erasures, trunc);
  for (uint32_t i = 0; i < GF_ORDER; i++) {
    uint32_t product = (uint32_t)erasures[i] * (uint32_t)g_log_walsh[i];
    erasures[i] = rso_add_mod(product & 0xFFFF, product >> 16);
  }
  rso_fwht(erasures, GF_ORDER);
}

/* -------------------------------------------------------------- root.zig */
static uint64_t ceil_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

/* root.zig:397-415. The reference asserts inside ceilPowerOfTwo(0) before its
 * own zero check; we return UnsupportedShardCount for 0 as line 406 intends. */
int rso_use_high_rate(uint64_t original, uint64_t recovery) {
  if (original > GF_ORDER || recovery > GF_ORDER) return -RSO_ERR_UNSUPPORTED_SHARD_COUNT;
  if (original == 0 || recovery == 0) return -RSO_ERR_UNSUPPORTED_SHARD_COUNT;
  uint64_t op = ceil_pow2(original), rp = ceil_pow2(recovery);
  uint64_t smaller = op < rp ? op : rp;
  uint64_t larger = original > recovery ? original : recovery;
  if (smaller + larger > GF_ORDER) return -RSO_ERR_UNSUPPORTED_SHARD_COUNT;
  if (op < rp) return 0;
  if (op > rp) return 1;
  return original <= recovery;
}

static int check_codec(uint64_t k, uint64_t m, size_t shard_bytes) {
  int hr = rso_use_high_rate(k, m);
  if (hr < 0) return -hr;
  if (hr == 0) return RSO_ERR_LOW_RATE_UNSUPPORTED; /* root.zig:120 @panic("TODO") */
  if (shard_bytes == 0 || (shard_bytes & 1)) return RSO_ERR_INVALID_SHARD_SIZE; /* root.zig:103 */
  /* shard_bytes % 64 != 0: the reference panics (root.zig:384-386); the oracle
   * implements the tail layout its undoLastChunkEncoding (root.zig:338-348) implies. */
  return RSO_OK;
}

/* Shards.insert (root.zig:373-387) for one shard of sb bytes into L = ceil(sb/64)
 * chunks. A tail of t bytes (t even, < 64) goes into the last chunk as
 * [0, t/2) -> lo bytes [0, t/2) and [t/2, t) -> hi bytes [32, 32 + t/2), the rest
 * zero — the inverse of undoLastChunkEncoding's memmove (root.zig:346). */
static void insert_shard(uint8_t *dst, const uint8_t *src, size_t sb) {
  const size_t whole = sb / 64 * 64, t = sb % 64;
  memcpy(dst, src, whole);
  if (t) {
    uint8_t *c = dst + whole;
    memset(c, 0, 64);
    memcpy(c, src + whole, t / 2);
    memcpy(c + 32, src + whole + t / 2, t / 2);
  }
}

/* copy out + undoLastChunkEncoding (root.zig:338-348, with the memmove applied to
 * the buffer itself rather than to a copy, defect D7) */
static void extract_shard(uint8_t *dst, const uint8_t *src, size_t sb) {
  const size_t whole = sb / 64 * 64, t = sb % 64;
  memcpy(dst, src, whole);
  if (t) {
    memcpy(dst + whole, src + whole, t / 2);
    memcpy(dst + whole + t / 2, src + whole + 32, t / 2);
  }
}

/* Encoder.encode on a prepared work buffer (root.zig:136-173).
 * work: [Wenc][L][64] with originals at positions 0..k, rest don't-care. */
static void encode_work(uint8_t *work, size_t L, uint64_t k, uint64_t m, int quirks) {
  uint64_t chunk = ceil_pow2(m);
  uint64_t first = k < chunk ? k : chunk;
  memset(SHARD(work, L, first), 0, (chunk - first) * L * 64); /* root.zig:145 */
  rso_ifft(work, L, 0, chunk, first, chunk, quirks);           /* root.zig:146 */
  if (k > chunk) {
    uint64_t cs = chunk;
    /* root.zig:151 — D2: the reference writes `<`, correct is `<=` */
    while ((quirks & RSO_Q_D2) ? (cs + chunk < k) : (cs + chunk <= k)) {
      rso_ifft(work, L, cs, chunk, chunk, cs + chunk, quirks);
      xor_chunks(work, SHARD(work, L, cs), chunk * L); /* D3 fixed: × L */
      cs += chunk;
    }
    uint64_t last = k % chunk; /* root.zig:159-166 */
    if (last > 0) {
      memset(SHARD(work, L, cs + last), 0, (chunk - last) * L * 64); /* D4 fixed */
      rso_ifft(work, L, cs, chunk, last, cs + chunk, quirks);
      xor_chunks(work, SHARD(work, L, cs), chunk * L);
    }
  }
  rso_fft(work, L, 0, chunk, m, 0, quirks); /* root.zig:169 */
}

/* top-level encode (root.zig:14-30) generalised to any even shard_bytes */
int rso_encode(uint64_t k, uint64_t m, size_t shard_bytes, const uint8_t *const *original,
               uint8_t *const *recovery_out, int quirks) {
  rso_init();
  if (k == 0 || original == NULL) return RSO_ERR_TOO_FEW_ORIGINAL_SHARDS;
  int st = check_codec(k, m, shard_bytes);
  if (st) return st;
  size_t L = (shard_bytes + 63) / 64; /* root.zig:115 divCeil */
  uint64_t chunk = ceil_pow2(m);
  uint64_t work_count = (k + chunk - 1) / chunk * chunk; /* root.zig:106 */
  uint8_t *work = calloc(work_count * L, 64);
  if (!work) return RSO_ERR_OUT_OF_MEMORY;
  for (uint64_t i = 0; i < k; i++) insert_shard(SHARD(work, L, i), original[i], shard_bytes); /* Shards.insert */
  encode_work(work, L, k, m, quirks);
  for (uint64_t r = 0; r < m; r++) extract_shard(recovery_out[r], SHARD(work, L, r), shard_bytes);
  free(work);
  return RSO_OK;
}

/* Low-rate encode (useHighRate == false). ABSENT from the reference
 * (root.zig:119-121 @panic("TODO")), so PARITY UNPINNED: restated from the
 * algorithm the reference ports, reed-solomon-simd's low-rate encoder
 * (benchmarks.zig:1-2 names the crate; it is not vendored here). Originals sit at
 * positions [0, k) of one chunk C = ceilPow2(k): IFFT(pos 0, size C, trunc k,
 * skew 0); recovery chunk j (shards [jC, jC + C)) = FFT of a copy of that chunk,
 * trunc min(C, m - jC), skew (j + 1)C — i.e. evaluations at positions [C, C + m). */
int rso_encode_low(uint64_t k, uint64_t m, size_t shard_bytes, const uint8_t *const *original,
                   uint8_t *const *recovery_out, int quirks) {
  rso_init();
  if (k == 0 || original == NULL) return RSO_ERR_TOO_FEW_ORIGINAL_SHARDS;
  int hr = rso_use_high_rate(k, m);
  if (hr < 0) return -hr;
  if (hr == 1) return RSO_ERR_UNSUPPORTED_SHARD_COUNT; /* high rate: rso_encode */
  if (shard_bytes == 0 || (shard_bytes & 1)) return RSO_ERR_INVALID_SHARD_SIZE;
  size_t L = (shard_bytes + 63) / 64;
  uint64_t C = ceil_pow2(k);
  uint8_t *coef = calloc(C * L, 64), *tmp = malloc(C * L * 64);
  if (!coef || !tmp) {
    free(coef);
    free(tmp);
    return RSO_ERR_OUT_OF_MEMORY;
  }
  for (uint64_t i = 0; i < k; i++) insert_shard(SHARD(coef, L, i), original[i], shard_bytes);
  rso_ifft(coef, L, 0, C, k, 0, quirks);
  for (uint64_t cs = 0; cs < m; cs += C) {
    uint64_t t = m - cs < C ? m - cs : C;
    memcpy(tmp, coef, C * L * 64);
    rso_fft(tmp, L, 0, C, t, cs + C, quirks);
    for (uint64_t i = 0; i < t; i++) extract_shard(recovery_out[cs + i], SHARD(tmp, L, i), shard_bytes);
  }
  free(coef);
  free(tmp);
  return RSO_OK;
}

/* Decoder.decode on a prepared work buffer (root.zig:268-335).
 * work: [Wdec][L][64]; received[pos] marks present positions (recovery at
 * [0,m), originals at [chunk, chunk+k)). Restored originals land in place. */
/* root.zig:277-289: the erasure flags of a received pattern -> evalPoly (logs) */
static void decode_erasures(uint64_t k, uint64_t m, const uint8_t *received, uint16_t *erasures) {
  uint64_t chunk = ceil_pow2(m);
  uint64_t original_end = chunk + k;
  memset(erasures, 0, GF_ORDER * sizeof(uint16_t));
  for (uint64_t i = 0; i < m; i++) /* root.zig:278-287 */
    if (!received[i]) erasures[i] = 1;
  for (uint64_t i = m; i < chunk; i++) erasures[i] = 1;
  for (uint64_t i = chunk; i < original_end; i++)
    if (!received[i]) erasures[i] = 1;
  rso_eval_poly(erasures, original_end); /* root.zig:289 */
}

/* the rest of Decoder.decode for erasures already evaluated (decode_erasures): a batch with
 * one erasure pattern evaluates the locator once, as a batched caller of the reference would */
static void decode_work_er(uint8_t *work, size_t L, uint64_t k, uint64_t m, const uint8_t *received,
                           const uint16_t *erasures, int quirks) {
  uint64_t chunk = ceil_pow2(m);
  uint64_t original_end = chunk + k;
  uint64_t work_count = ceil_pow2(chunk + k);
  for (uint64_t i = 0; i < m; i++) {     /* root.zig:292-303 */
    if (received[i]) rso_mul_scalar(SHARD(work, L, i), L, erasures[i], quirks);
    else memset(SHARD(work, L, i), 0, L * 64);
  }
  memset(SHARD(work, L, m), 0, (chunk - m) * L * 64);
  for (uint64_t i = chunk; i < original_end; i++) {
    if (received[i]) rso_mul_scalar(SHARD(work, L, i), L, erasures[i], quirks);
    else memset(SHARD(work, L, i), 0, L * 64);
  }
  memset(SHARD(work, L, original_end), 0, (work_count - original_end) * L * 64); /* D4 fixed */
  rso_ifft(work, L, 0, work_count, original_end, 0, quirks);                    /* root.zig:306 */
  for (uint64_t i = 1; i < work_count; i++) {                                   /* root.zig:309-315 */
    uint64_t width = 1ull << __builtin_ctzll(i);
    xor_chunks(SHARD(work, L, i - width), SHARD(work, L, i), width * L); /* D5 fixed */
  }
  rso_fft(work, L, 0, work_count, original_end, 0, quirks); /* root.zig:318 */
  for (uint64_t i = chunk; i < original_end; i++)          /* root.zig:321-326 */
    if (!received[i]) rso_mul_scalar(SHARD(work, L, i), L, (uint16_t)(GF_MODULUS - erasures[i]), quirks);
}

static void decode_work(uint8_t *work, size_t L, uint64_t k, uint64_t m, const uint8_t *received,
                        uint16_t *erasures, int quirks) {
  decode_erasures(k, m, received, erasures);
  decode_work_er(work, L, k, m, received, erasures, quirks);
}

/* top-level decode (root.zig:32-84) generalised to any even shard_bytes */
int rso_decode(uint64_t k, uint64_t m, size_t shard_bytes, const uint8_t *const *original,
               const uint8_t *const *recovery, uint8_t *const *restored_out, int quirks) {
  rso_init();
  uint64_t orig_present = 0, rec_present = 0;
  for (uint64_t i = 0; i < k; i++) orig_present += original[i] != NULL;
  for (uint64_t i = 0; i < m; i++) rec_present += recovery[i] != NULL;
  if (rec_present == 0) { /* root.zig:42-58 */
    if (orig_present != k) return RSO_ERR_NOT_ENOUGH_SHARDS;
    for (uint64_t i = 0; i < k; i++) memcpy(restored_out[i], original[i], shard_bytes);
    return RSO_OK;
  }
  int st = check_codec(k, m, shard_bytes);
  if (st) return st;
  if (orig_present + rec_present < k) return RSO_ERR_NOT_ENOUGH_SHARDS; /* root.zig:271 */
  size_t L = (shard_bytes + 63) / 64;
  uint64_t chunk = ceil_pow2(m);
  uint64_t work_count = ceil_pow2(chunk + k); /* root.zig:204 */
  uint8_t *work = calloc(work_count * L, 64);
  uint8_t *received = calloc(work_count, 1);
  uint16_t *erasures = malloc(GF_ORDER * sizeof(uint16_t));
  if (!work || !received || !erasures) {
    free(work);
    free(received);
    free(erasures);
    return RSO_ERR_OUT_OF_MEMORY;
  }
  for (uint64_t i = 0; i < k; i++)
    if (original[i]) {
      insert_shard(SHARD(work, L, chunk + i), original[i], shard_bytes);
      received[chunk + i] = 1;
    }
  for (uint64_t i = 0; i < m; i++)
    if (recovery[i]) {
      insert_shard(SHARD(work, L, i), recovery[i], shard_bytes);
      received[i] = 1;
    }
  decode_work(work, L, k, m, received, erasures, quirks);
  for (uint64_t i = 0; i < k; i++) /* root.zig:76-81 */
    if (original[i]) memcpy(restored_out[i], original[i], shard_bytes);
    else extract_shard(restored_out[i], SHARD(work, L, chunk + i), shard_bytes);
  free(work);
  free(received);
  free(erasures);
  return RSO_OK;
}

/* ------------------------------------------------------- batched, threaded */
typedef struct {
  int op; /* 0 encode, 1 reconstruct */
  uint64_t k, m;
  size_t shard_bytes, s_begin, s_end;
  const uint8_t *in;
  uint8_t *out;
  const uint8_t *present;
  int quirks;
  int status;
} batch_job;

static void *batch_worker(void *arg) {
  batch_job *j = arg;
  size_t L = (j->shard_bytes + 63) / 64, sb = j->shard_bytes;
  uint64_t k = j->k, m = j->m, chunk = ceil_pow2(m);
  if (j->op == 0) {
    uint64_t wc = (k + chunk - 1) / chunk * chunk;
    uint8_t *work = calloc(wc * L, 64); /* Encoder.init: untimed in the reference harness */
    if (!work) {
      j->status = RSO_ERR_OUT_OF_MEMORY;
      return NULL;
    }
    for (size_t s = j->s_begin; s < j->s_end; s++) {
      const uint8_t *src = j->in + s * k * sb;
      for (uint64_t i = 0; i < k; i++) insert_shard(SHARD(work, L, i), src + i * sb, sb); /* addOriginalShard x k */
      encode_work(work, L, k, m, j->quirks);
      for (uint64_t r = 0; r < m; r++) extract_shard(j->out + (s * m + r) * sb, SHARD(work, L, r), sb);
    }
    free(work);
  } else {
    uint64_t wc = ceil_pow2(chunk + k);
    uint8_t *work = calloc(wc * L, 64);
    uint8_t *received = calloc(wc, 1);
    uint16_t *erasures = malloc(GF_ORDER * sizeof(uint16_t));
    uint64_t e = 0;
    for (uint64_t i = 0; i < k; i++) e += !j->present[i];
    for (uint64_t i = 0; i < k; i++) received[chunk + i] = j->present[i] != 0;
    for (uint64_t i = 0; i < m; i++) received[i] = j->present[k + i] != 0;
    decode_erasures(k, m, received, erasures); /* one pattern for the whole batch */
    for (size_t s = j->s_begin; s < j->s_end; s++) {
      const uint8_t *src = j->in + s * (k + m) * sb;
      for (uint64_t i = 0; i < k; i++)
        if (j->present[i]) insert_shard(SHARD(work, L, chunk + i), src + i * sb, sb);
      for (uint64_t i = 0; i < m; i++)
        if (j->present[k + i]) insert_shard(SHARD(work, L, i), src + (k + i) * sb, sb);
      decode_work_er(work, L, k, m, received, erasures, j->quirks);
      uint64_t o = 0;
      for (uint64_t i = 0; i < k; i++)
        if (!j->present[i]) extract_shard(j->out + (s * e + o++) * sb, SHARD(work, L, chunk + i), sb);
    }
    free(work);
    free(received);
    free(erasures);
  }
  j->status = RSO_OK;
  return NULL;
}

static int run_batch(batch_job proto, size_t n_stripes, int threads) {
  if (threads < 1) threads = 1;
  if ((size_t)threads > n_stripes) threads = (int)(n_stripes ? n_stripes : 1);
  batch_job *jobs = calloc((size_t)threads, sizeof *jobs);
  pthread_t *tids = calloc((size_t)threads, sizeof *tids);
  size_t per = (n_stripes + threads - 1) / threads;
  for (int t = 0; t < threads; t++) {
    jobs[t] = proto;
    jobs[t].s_begin = t * per < n_stripes ? t * per : n_stripes;
    jobs[t].s_end = (t + 1) * per < n_stripes ? (t + 1) * per : n_stripes;
    if (threads == 1) batch_worker(&jobs[t]);
    else pthread_create(&tids[t], NULL, batch_worker, &jobs[t]);
  }
  int st = RSO_OK;
  for (int t = 0; t < threads; t++) {
    if (threads > 1) pthread_join(tids[t], NULL);
    if (jobs[t].status) st = jobs[t].status;
  }
  free(jobs);
  free(tids);
  return st;
}

int rso_encode_batch(uint64_t k, uint64_t m, size_t shard_bytes, size_t n_stripes, const uint8_t *data,
                     uint8_t *parity, int quirks, int threads) {
  rso_init();
  int st = check_codec(k, m, shard_bytes);
  if (st) return st;
  batch_job p = {0};
  p.op = 0;
  p.k = k;
  p.m = m;
  p.shard_bytes = shard_bytes;
  p.in = data;
  p.out = parity;
  p.quirks = quirks;
  return run_batch(p, n_stripes, threads);
}

int rso_reconstruct_batch(uint64_t k, uint64_t m, size_t shard_bytes, size_t n_stripes, const uint8_t *present,
                          const uint8_t *shards, uint8_t *restored, int quirks, int threads) {
  rso_init();
  int st = check_codec(k, m, shard_bytes);
  if (st) return st;
  uint64_t have = 0;
  for (uint64_t i = 0; i < k + m; i++) have += present[i] != 0;
  if (have < k) return RSO_ERR_NOT_ENOUGH_SHARDS;
  batch_job p = {0};
  p.op = 1;
  p.k = k;
  p.m = m;
  p.shard_bytes = shard_bytes;
  p.in = shards;
  p.out = restored;
  p.present = present;
  p.quirks = quirks;
  return run_batch(p, n_stripes, threads);
}

/* benchmarks.zig:14-61 protocol, natively: mean ns per encode of k originals of
 * shard_bytes random bytes (insert + encode timed; the work buffer is allocated
 * outside the timed region, like the reference's untimed Encoder.init). */
double rso_bench_encode(uint64_t k, uint64_t m, size_t shard_bytes, uint64_t iters, int quirks) {
  rso_init();
  if (check_codec(k, m, shard_bytes)) return -1.0;
  size_t L = (shard_bytes + 63) / 64;
  uint64_t chunk = ceil_pow2(m);
  uint64_t work_count = (k + chunk - 1) / chunk * chunk;
  uint8_t *orig = malloc(k * shard_bytes), *work = calloc(work_count * L, 64);
  if (!orig || !work) {
    free(orig);
    free(work);
    return -1.0;
  }
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (size_t i = 0; i < k * shard_bytes; i++) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    orig[i] = (uint8_t)x;
  }
  struct timespec a, b;
  double total = 0;
  for (uint64_t it = 0; it < iters; it++) {
    memset(work, 0, work_count * L * 64); /* Shards.init zeroes (untimed) */
    clock_gettime(CLOCK_MONOTONIC, &a);
    for (uint64_t i = 0; i < k; i++) insert_shard(SHARD(work, L, i), orig + i * shard_bytes, shard_bytes);
    encode_work(work, L, k, m, quirks);
    clock_gettime(CLOCK_MONOTONIC, &b);
    total += (double)(b.tv_sec - a.tv_sec) * 1e9 + (double)(b.tv_nsec - a.tv_nsec);
  }
  free(orig);
  free(work);
  return total / (double)iters;
}
