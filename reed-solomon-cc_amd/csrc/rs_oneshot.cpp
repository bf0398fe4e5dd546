// rs_oneshot.cpp — one-shot host API (root.zig:14-84), Encoder / Decoder objects
// (root.zig:86-336) and the Engine seam test shims (Generic.zig).
#include "rs_host.hpp"

using namespace rs;
using namespace rs::host;

// ------------------------------------------------------------ one-shot host
namespace {
struct DevMem {
  void *p = nullptr;
  ~DevMem() {
    if (p) (void)hipFree(p);
  }
};

// One-shot calls (rs_encode / rs_decode and the Encoder / Decoder objects, root.zig:14-84)
// move one stripe: a pooled context per call in flight holds a pinned host buffer, a
// device buffer and a stream, so a call packs its shards into pinned memory and makes
// one H2D copy, the kernel and one D2H copy with a single synchronisation (instead of
// two hipMallocs and k + m synchronous copies). Contexts are kept for reuse (never freed:
// process-lifetime, like the plan caches' device tables).
struct OneShot {
  int dev = -1;
  hipStream_t s = nullptr;
  uint8_t *h = nullptr, *d = nullptr;
  size_t bytes = 0;
};
std::mutex g_oneshot_mu;
std::vector<OneShot *> g_oneshot_free;

int oneshot_acquire(int dev, size_t bytes, OneShot **out) {
  OneShot *c = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_oneshot_mu);
    for (size_t i = 0; i < g_oneshot_free.size(); i++)
      if (g_oneshot_free[i]->dev == dev) {
        c = g_oneshot_free[i];
        g_oneshot_free.erase(g_oneshot_free.begin() + static_cast<std::ptrdiff_t>(i));
        break;
      }
  }
  if (!c) {
    alloc_point();
    c = new OneShot;
    c->dev = dev;
    hipError_t e = hipStreamCreateWithFlags(&c->s, hipStreamNonBlocking);
    if (e != hipSuccess) {
      delete c;
      return hip_fail(e, "hipStreamCreateWithFlags");
    }
  }
  if (c->bytes < bytes) {  // grow to the next power of two
    size_t nb = 1 << 16;
    while (nb < bytes) nb <<= 1;
    if (c->h) (void)hipHostFree(c->h);
    if (c->d) (void)hipFree(c->d);
    c->h = c->d = nullptr;
    c->bytes = 0;
    hipError_t e = pinned_malloc(reinterpret_cast<void **>(&c->h), nb);
    if (e == hipSuccess) e = dev_malloc(reinterpret_cast<void **>(&c->d), nb);
    if (e != hipSuccess) {
      if (c->h) (void)hipHostFree(c->h);
      c->h = nullptr;
      std::lock_guard<std::mutex> lk(g_oneshot_mu);
      g_oneshot_free.push_back(c);
      return hip_fail(e, "one-shot staging buffers");
    }
    c->bytes = nb;
  }
  *out = c;
  return RS_OK;
}

void oneshot_release(OneShot *c) {
  std::lock_guard<std::mutex> lk(g_oneshot_mu);
  g_oneshot_free.push_back(c);
}

struct OneShotLease {  // drains the stream and returns the context on every exit path
  OneShot *c = nullptr;
  ~OneShotLease() {
    if (c) {
      (void)hipStreamSynchronize(c->s);
      oneshot_release(c);
    }
  }
};

inline size_t align256(size_t x) { return (x + 255) & ~static_cast<size_t>(255); }
}  // namespace

void rs::host::release_oneshot() {
  std::vector<OneShot *> all;
  {
    std::lock_guard<std::mutex> lk(g_oneshot_mu);
    all.swap(g_oneshot_free);  // contexts leased by calls in flight come back later
  }
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (OneShot *c : all) {
    (void)hipSetDevice(c->dev);
    if (c->h) (void)hipHostFree(c->h);
    if (c->d) (void)hipFree(c->d);
    if (c->s) (void)hipStreamDestroy(c->s);
    delete c;
  }
  (void)hipSetDevice(cur);
}

size_t rs::host::oneshot_pooled() {
  std::lock_guard<std::mutex> lk(g_oneshot_mu);
  return g_oneshot_free.size();
}

extern "C" {

int rs_encode(uint64_t k, uint64_t m, size_t sb, const uint8_t *const *original, uint8_t *const *recovery_out) {
  TraceScope ts;
  return guarded([&]() -> int {
    if (k == 0 || !original) return fail(RS_ERR_TOO_FEW_ORIGINAL_SHARDS, "no original shards");  // root.zig:20
    int st = check_codec(k, m, sb);
    if (st) return st;
    for (uint64_t i = 0; i < k; i++)
      if (!original[i]) return fail(RS_ERR_INVALID_ARGUMENT, "NULL original shard");
    if (!recovery_out) return fail(RS_ERR_INVALID_ARGUMENT, "NULL recovery_out");
    int dev;
    if ((st = current_device(&dev))) return st;
    const size_t off = align256(k * sb);
    OneShotLease lease;
    if ((st = oneshot_acquire(dev, off + m * sb, &lease.c))) return st;
    OneShot &c = *lease.c;
    for (uint64_t i = 0; i < k; i++) std::memcpy(c.h + i * sb, original[i], sb);
    HIP_TRY(hipMemcpyAsync(c.d, c.h, k * sb, hipMemcpyHostToDevice, c.s));
    st = rs_encode_batch_dev(k, m, sb, 1, c.d, 0, c.d + off, 0, RS_FLAG_CORRECTED, c.s);
    if (st == RS_OK) HIP_TRY(hipMemcpyAsync(c.h + off, c.d + off, m * sb, hipMemcpyDeviceToHost, c.s));
    HIP_TRY(hipStreamSynchronize(c.s));  // also drains a failed call's queued copy
    if (st) return st;
    for (uint64_t r = 0; r < m; r++) std::memcpy(recovery_out[r], c.h + off + r * sb, sb);
    return RS_OK;
  });
}

int rs_decode(uint64_t k, uint64_t m, size_t sb, const uint8_t *const *original, const uint8_t *const *recovery,
              uint8_t *const *restored_out) {
  TraceScope ts;
  return guarded([&]() -> int {
    if (!original || !recovery || !restored_out) return fail(RS_ERR_INVALID_ARGUMENT, "NULL array");
    uint64_t orig_present = 0, rec_present = 0;
    for (uint64_t i = 0; i < k; i++) orig_present += original[i] != nullptr;
    for (uint64_t i = 0; i < m; i++) rec_present += recovery[i] != nullptr;
    if (rec_present == 0) {  // root.zig:39-59
      if (orig_present != k) return fail(RS_ERR_NOT_ENOUGH_SHARDS, "no recovery shards and originals incomplete");
      for (uint64_t i = 0; i < k; i++) std::memcpy(restored_out[i], original[i], sb);
      return RS_OK;
    }
    int st = check_codec(k, m, sb);
    if (st) return st;
    if (orig_present + rec_present < k) return fail(RS_ERR_NOT_ENOUGH_SHARDS, "not enough shards");  // root.zig:271
    std::vector<uint8_t> present(k + m);
    for (uint64_t i = 0; i < k; i++) present[i] = original[i] != nullptr;
    for (uint64_t i = 0; i < m; i++) present[k + i] = recovery[i] != nullptr;
    const uint64_t e = k - orig_present;
    if (e > 0) {
      int dev;
      if ((st = current_device(&dev))) return st;
      // staging: [originals k][recovery m][restored e], each region 256-B aligned; absent
      // slots are not filled (the kernels never read them)
      const size_t o_rec = align256(k * sb), o_out = o_rec + align256(m * sb);
      OneShotLease lease;
      if ((st = oneshot_acquire(dev, o_out + e * sb, &lease.c))) return st;
      OneShot &c = *lease.c;
      for (uint64_t i = 0; i < k; i++)
        if (original[i]) std::memcpy(c.h + i * sb, original[i], sb);
      for (uint64_t i = 0; i < m; i++)
        if (recovery[i]) std::memcpy(c.h + o_rec + i * sb, recovery[i], sb);
      HIP_TRY(hipMemcpyAsync(c.d, c.h, o_rec + m * sb, hipMemcpyHostToDevice, c.s));
      st = rs_reconstruct_batch_dev(k, m, sb, 1, present.data(), c.d, 0, c.d + o_rec, 0, c.d + o_out, 0,
                                    RS_FLAG_CORRECTED, c.s);
      if (st == RS_OK) HIP_TRY(hipMemcpyAsync(c.h + o_out, c.d + o_out, e * sb, hipMemcpyDeviceToHost, c.s));
      HIP_TRY(hipStreamSynchronize(c.s));
      if (st) return st;
      uint64_t slot = 0;
      for (uint64_t i = 0; i < k; i++)
        if (!original[i]) std::memcpy(restored_out[i], c.h + o_out + (slot++) * sb, sb);
    }
    for (uint64_t i = 0; i < k; i++)  // root.zig:76-81
      if (original[i]) std::memcpy(restored_out[i], original[i], sb);
    return RS_OK;
  });
}

// ---------------------------------------------------------------- Encoder
struct rs_encoder {
  uint64_t k, m;
  size_t sb;
  uint64_t received = 0;
  std::vector<uint8_t> originals, recovery;
};

int rs_encoder_new(uint64_t k, uint64_t m, size_t sb, rs_encoder **out) {
  return guarded([&]() -> int {
    if (!out) return fail(RS_ERR_INVALID_ARGUMENT, "out == NULL");
    *out = nullptr;
    int st = check_codec(k, m, sb);  // root.zig:100-103
    if (st) return st;
    try {
      alloc_point();
      rs_encoder *e = new rs_encoder;
      e->k = k;
      e->m = m;
      e->sb = sb;
      e->originals.assign(k * sb, 0);
      e->recovery.assign(m * sb, 0);
      *out = e;
    } catch (...) {
      return fail(RS_ERR_OUT_OF_MEMORY, "allocation failed");
    }
    return RS_OK;
  });
}

int rs_encoder_add_original_shard(rs_encoder *e, const uint8_t *shard, size_t len) {
  return guarded([&]() -> int {
    if (!e || !shard) return fail(RS_ERR_INVALID_ARGUMENT, "NULL argument");
    if (e->received == e->k) return fail(RS_ERR_TOO_MANY_ORIGINAL_SHARDS, "too many original shards");  // root.zig:129
    if (len != e->sb) return fail(RS_ERR_DIFFERENT_SHARD_SIZE, "shard length differs");                // root.zig:130
    std::memcpy(e->originals.data() + e->received * e->sb, shard, len);
    e->received++;
    return RS_OK;
  });
}

int rs_encoder_encode(rs_encoder *e, const uint8_t **recovery_out) {
  TraceScope ts;
  return guarded([&]() -> int {
    if (!e) return fail(RS_ERR_INVALID_ARGUMENT, "NULL encoder");
    if (e->received != e->k) return fail(RS_ERR_TOO_FEW_ORIGINAL_SHARDS, "too few original shards");  // root.zig:139
    std::vector<const uint8_t *> in(e->k);
    std::vector<uint8_t *> out(e->m);
    for (uint64_t i = 0; i < e->k; i++) in[i] = e->originals.data() + i * e->sb;
    for (uint64_t i = 0; i < e->m; i++) out[i] = e->recovery.data() + i * e->sb;
    int st = rs_encode(e->k, e->m, e->sb, in.data(), out.data());
    if (st) return st;
    if (recovery_out)
      for (uint64_t i = 0; i < e->m; i++) recovery_out[i] = out[i];
    return RS_OK;
  });
}

int rs_encoder_reset(rs_encoder *e) {
  return guarded([&]() -> int {
    if (!e) return fail(RS_ERR_INVALID_ARGUMENT, "NULL encoder");
    e->received = 0;
    return RS_OK;
  });
}

void rs_encoder_free(rs_encoder *e) { delete e; }

// ---------------------------------------------------------------- Decoder
struct rs_decoder {
  uint64_t k, m;
  size_t sb;
  uint64_t orig_received = 0, rec_received = 0;
  std::vector<uint8_t> originals, recovery, restored;
  std::vector<uint8_t> have_orig, have_rec;
};

int rs_decoder_new(uint64_t k, uint64_t m, size_t sb, rs_decoder **out) {
  return guarded([&]() -> int {
    if (!out) return fail(RS_ERR_INVALID_ARGUMENT, "out == NULL");
    *out = nullptr;
    int st = check_codec(k, m, sb);  // root.zig:198-201
    if (st) return st;
    try {
      alloc_point();
      rs_decoder *d = new rs_decoder;
      d->k = k;
      d->m = m;
      d->sb = sb;
      d->originals.assign(k * sb, 0);
      d->recovery.assign(m * sb, 0);
      d->restored.assign(k * sb, 0);
      d->have_orig.assign(k, 0);
      d->have_rec.assign(m, 0);
      *out = d;
    } catch (...) {
      return fail(RS_ERR_OUT_OF_MEMORY, "allocation failed");
    }
    return RS_OK;
  });
}

// root.zig:236-248
int rs_decoder_add_original_shard(rs_decoder *d, uint64_t index, const uint8_t *shard, size_t len) {
  return guarded([&]() -> int {
    if (!d || !shard) return fail(RS_ERR_INVALID_ARGUMENT, "NULL argument");
    if (index >= d->k) return fail(RS_ERR_INVALID_SHARD_INDEX, "original index out of range");
    if (d->have_orig[index]) return fail(RS_ERR_DUPLICATE_SHARD_INDEX, "duplicate original index");
    if (d->orig_received == d->k) return fail(RS_ERR_TOO_MANY_SHARDS, "too many original shards");
    if (len != d->sb) return fail(RS_ERR_DIFFERENT_SHARD_SIZE, "shard length differs");
    std::memcpy(d->originals.data() + index * d->sb, shard, len);
    d->have_orig[index] = 1;
    d->orig_received++;
    return RS_OK;
  });
}

// root.zig:250-265
int rs_decoder_add_recovery_shard(rs_decoder *d, uint64_t index, const uint8_t *shard, size_t len) {
  return guarded([&]() -> int {
    if (!d || !shard) return fail(RS_ERR_INVALID_ARGUMENT, "NULL argument");
    if (index >= d->m) return fail(RS_ERR_INVALID_SHARD_INDEX, "recovery index out of range");
    if (d->have_rec[index]) return fail(RS_ERR_DUPLICATE_SHARD_INDEX, "duplicate recovery index");
    if (d->rec_received == d->m) return fail(RS_ERR_TOO_MANY_SHARDS, "too many recovery shards");
    if (len != d->sb) return fail(RS_ERR_DIFFERENT_SHARD_SIZE, "shard length differs");
    std::memcpy(d->recovery.data() + index * d->sb, shard, len);
    d->have_rec[index] = 1;
    d->rec_received++;
    return RS_OK;
  });
}

// root.zig:268-335; restored_out[i] points at the original (supplied or restored)
int rs_decoder_decode(rs_decoder *d, const uint8_t **restored_out) {
  TraceScope ts;
  return guarded([&]() -> int {
    if (!d) return fail(RS_ERR_INVALID_ARGUMENT, "NULL decoder");
    if (d->orig_received + d->rec_received < d->k) return fail(RS_ERR_NOT_ENOUGH_SHARDS, "not enough shards");
    std::vector<const uint8_t *> o(d->k), r(d->m);
    std::vector<uint8_t *> out(d->k);
    for (uint64_t i = 0; i < d->k; i++) {
      o[i] = d->have_orig[i] ? d->originals.data() + i * d->sb : nullptr;
      out[i] = d->restored.data() + i * d->sb;
    }
    for (uint64_t i = 0; i < d->m; i++) r[i] = d->have_rec[i] ? d->recovery.data() + i * d->sb : nullptr;
    int st = rs_decode(d->k, d->m, d->sb, o.data(), r.data(), out.data());
    if (st) return st;
    if (restored_out)
      for (uint64_t i = 0; i < d->k; i++) restored_out[i] = out[i];
    return RS_OK;
  });
}

void rs_decoder_free(rs_decoder *d) { delete d; }

// ------------------------------------------------------------- engine shims
static int engine_transform(uint8_t *shards, uint64_t count, size_t sb, uint64_t pos, uint64_t size,
                            uint64_t trunc, uint64_t sd, uint32_t flags, bool inverse) {
  if (!shards) return fail(RS_ERR_INVALID_ARGUMENT, "NULL shards");
  if (sb == 0 || sb % 64) return fail(RS_ERR_INVALID_SHARD_SIZE, "shard_bytes must be a multiple of 64");
  if (pos + size > count || trunc > size) return fail(RS_ERR_INVALID_ARGUMENT, "pos/size/trunc out of range");
  int dev, st;
  if ((st = current_device(&dev))) return st;
  std::vector<RsTab> tabs;
  if (inverse) push_ifft_tabs(tabs, size, sd, flags & RS_FLAG_QUIRK_D1);
  else push_fft_tabs(tabs, size, sd, flags & RS_FLAG_QUIRK_D1);
  DevMem dt, dw;
  HIP_TRY(dev_malloc(&dt.p, std::max<size_t>(16, tabs.size() * sizeof(RsTab))));
  if (!tabs.empty()) HIP_TRY(hipMemcpy(dt.p, tabs.data(), tabs.size() * sizeof(RsTab), hipMemcpyHostToDevice));
  HIP_TRY(dev_malloc(&dw.p, count * sb));
  HIP_TRY(hipMemcpy(dw.p, shards, count * sb, hipMemcpyHostToDevice));
  HIP_TRY(launch_engine_fft(static_cast<uint8_t *>(dw.p), sb, pos, size, trunc, static_cast<const RsTab *>(dt.p),
                            inverse, nullptr));
  HIP_TRY(hipMemcpy(shards, dw.p, count * sb, hipMemcpyDeviceToHost));
  return RS_OK;
}

int rs_engine_fft(uint8_t *shards, uint64_t count, size_t sb, uint64_t pos, uint64_t size, uint64_t trunc,
                  uint64_t sd, uint32_t flags) {
  TraceScope ts;
  return guarded([&]() -> int {
    return engine_transform(shards, count, sb, pos, size, trunc, sd, flags, false);
  });
}

int rs_engine_ifft(uint8_t *shards, uint64_t count, size_t sb, uint64_t pos, uint64_t size, uint64_t trunc,
                   uint64_t sd, uint32_t flags) {
  TraceScope ts;
  return guarded([&]() -> int {
    return engine_transform(shards, count, sb, pos, size, trunc, sd, flags, true);
  });
}

int rs_engine_mul_scalar(uint8_t *chunks, size_t bytes, uint16_t log_m, uint32_t flags) {
  TraceScope ts;
  return guarded([&]() -> int {
    if (!chunks) return fail(RS_ERR_INVALID_ARGUMENT, "NULL chunks");
    if (bytes == 0 || bytes % 64) return fail(RS_ERR_INVALID_SHARD_SIZE, "bytes must be a multiple of 64");
    int dev, st;
    if ((st = current_device(&dev))) return st;
    const RsTab t = make_tab(log_m, flags & RS_FLAG_QUIRK_D1);
    DevMem dt, dw;
    HIP_TRY(dev_malloc(&dt.p, sizeof t));
    HIP_TRY(hipMemcpy(dt.p, &t, sizeof t, hipMemcpyHostToDevice));
    HIP_TRY(dev_malloc(&dw.p, bytes));
    HIP_TRY(hipMemcpy(dw.p, chunks, bytes, hipMemcpyHostToDevice));
    HIP_TRY(launch_mul_scalar(static_cast<uint8_t *>(dw.p), bytes, static_cast<const RsTab *>(dt.p), nullptr));
    HIP_TRY(hipMemcpy(chunks, dw.p, bytes, hipMemcpyDeviceToHost));
    return RS_OK;
  });
}

int rs_engine_eval_poly(uint16_t *erasures, uint64_t trunc) {
  TraceScope ts;
  return guarded([&]() -> int {
    if (!erasures) return fail(RS_ERR_INVALID_ARGUMENT, "NULL erasures");
    if (trunc > kOrder) return fail(RS_ERR_INVALID_ARGUMENT, "truncated_size > 65536");
    eval_poly(erasures, trunc);
    return RS_OK;
  });
}

}  // extern "C"
