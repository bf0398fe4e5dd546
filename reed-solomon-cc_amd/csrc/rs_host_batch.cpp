// rs_host_batch.cpp — host-resident batches (end to end through a persistent 2-slot
// H2D -> kernel -> D2H ring per device) and their multi-GPU split.
#include <cstdint>
#include <cstring>
#include <thread>
#include <utility>
#include <vector>

#include "rs_host.hpp"

using namespace rs;
using namespace rs::host;

extern "C" int rs_encode_batch_dev(uint64_t, uint64_t, size_t, uint64_t, const void *, uint64_t, void *, uint64_t,
                                   uint32_t, rs_stream_t);
extern "C" int rs_reconstruct_batch_dev(uint64_t, uint64_t, size_t, uint64_t, const uint8_t *, const void *, uint64_t,
                                        const void *, uint64_t, void *, uint64_t, uint32_t, rs_stream_t);

namespace {

// Copy `rows` rows of `row_bytes` between (possibly strided) buffers, always in the 2D form: for
// pinned host memory it moves contiguous slices faster than hipMemcpyAsync does (RS(10,4) 1 MiB
// encode 41.5 -> 52.3 GiB/s of data, 62 -> 79 GB/s over PCIe; c4 encode 44.6 -> 52.4;
// profiles/r06/e2e/copy2d/). RS_AMD_HOST_COPY2D=0 sends contiguous copies as hipMemcpyAsync.
bool copy_2d_always() {
  const char *e = std::getenv("RS_AMD_HOST_COPY2D");
  return !(e && *e == '0');
}
hipError_t copy_rows(void *dst, uint64_t dst_stride, const void *src, uint64_t src_stride, uint64_t row_bytes,
                     uint64_t rows, hipMemcpyKind kind, hipStream_t s) {
  if (rows == 0 || row_bytes == 0) return hipSuccess;
  if (dst_stride == row_bytes && src_stride == row_bytes && !copy_2d_always())
    return hipMemcpyAsync(dst, src, rows * row_bytes, kind, s);
  return hipMemcpy2DAsync(dst, dst_stride, src, src_stride, row_bytes, rows, kind, s);
}

// Pageable host buffers go through the ring's own pinned staging (RS_AMD_HOST_STAGE, default
// on): host threads copy a slice's rows into it while the previous slice is on PCIe, and the
// device copies run from pinned memory in the 2D form; the runtime's own pageable path stages
// through a smaller buffer one copy at a time.
bool host_stage_on() {
  const char *e = std::getenv("RS_AMD_HOST_STAGE");
  return !(e && *e == '0');
}
bool is_pinned(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost || a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged ||
         a.type == hipMemoryTypeUnified;
}
int stage_threads() {
  const char *e = std::getenv("RS_AMD_HOST_THREADS");
  const int hw = static_cast<int>(std::thread::hardware_concurrency());
  return e && *e ? std::max(1, std::min(64, std::atoi(e))) : std::max(1, std::min(16, hw));
}
// strided host-to-host copies (rows of `w` bytes), split into <= 4 MiB pieces over host threads
struct CopyJob {
  uint8_t *d;
  uint64_t ds;
  const uint8_t *s;
  uint64_t ss, w, rows;
};
void host_copy(const std::vector<CopyJob> &jobs) {
  struct Piece {
    uint8_t *d;
    const uint8_t *s;
    uint64_t len;
  };
  std::vector<Piece> pieces;
  for (const CopyJob &j : jobs)
    for (uint64_t r = 0; r < j.rows; r++)
      for (uint64_t o = 0; o < j.w; o += 4ull << 20)
        pieces.push_back({j.d + r * j.ds + o, j.s + r * j.ss + o, std::min<uint64_t>(4ull << 20, j.w - o)});
  const int T = static_cast<int>(std::min<uint64_t>(static_cast<uint64_t>(stage_threads()), pieces.size()));
  auto work = [&](int t) {
    for (size_t i = static_cast<size_t>(t); i < pieces.size(); i += static_cast<size_t>(T))
      std::memcpy(pieces[i].d, pieces[i].s, pieces[i].len);
  };
  if (T <= 1) {
    if (T == 1) work(0);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T - 1);
  for (int t = 1; t < T; t++) th.emplace_back(work, t);
  work(0);
  for (auto &x : th) x.join();
}

// Per-device staging ring of the host-batch calls: `slots` slices, each on its own
// stream (H2D -> kernel -> D2H in order; slices on different streams overlap both
// PCIe directions with the kernels). Buffers and streams persist across calls and
// grow on demand; the ring's mutex serialises host-batch calls on one device.
struct Pipeline {
  static constexpr int kMaxSlots = 8;
  std::mutex mu;
  int slots = 0;  // ring depth in use (RS_AMD_HOST_SLOTS, default 2)
  hipStream_t st[kMaxSlots] = {};
  void *buf[kMaxSlots][3] = {};
  uint64_t cap[3] = {};
  void *hst[kMaxSlots][3] = {};  // pinned host staging of pageable callers' slices
  uint64_t hcap[3] = {};
  int hslots = 0;
  int ensure_stage(const uint64_t bytes[3], int want) {
    bool grow = want > hslots;
    for (int j = 0; j < 3; j++) grow = grow || bytes[j] > hcap[j];
    if (!grow) return RS_OK;
    for (int i = 0; i < kMaxSlots; i++)
      for (int j = 0; j < 3; j++) {
        if (hst[i][j]) HIP_TRY(hipHostFree(hst[i][j]));
        hst[i][j] = nullptr;
      }
    hslots = 0;
    for (int j = 0; j < 3; j++) hcap[j] = std::max(hcap[j], bytes[j]);
    for (int i = 0; i < want; i++)
      for (int j = 0; j < 3; j++)
        if (hcap[j]) HIP_TRY(pinned_malloc(&hst[i][j], hcap[j]));
    hslots = want;
    return RS_OK;
  }
  int ensure(const uint64_t bytes[3], int want) {
    for (int i = 0; i < want; i++)
      if (!st[i]) HIP_TRY(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    bool grow = want > slots;  // fewer slots wanted: the call uses the first `want`
    for (int j = 0; j < 3; j++) grow = grow || bytes[j] > cap[j];
    if (!grow) return RS_OK;
    for (int i = 0; i < kMaxSlots; i++)
      for (int j = 0; j < 3; j++) {
        if (buf[i][j]) HIP_TRY(hipFree(buf[i][j]));
        buf[i][j] = nullptr;
      }
    slots = 0;
    for (int j = 0; j < 3; j++) cap[j] = std::max(cap[j], bytes[j]);
    for (int i = 0; i < want; i++)
      for (int j = 0; j < 3; j++)
        if (cap[j]) HIP_TRY(dev_malloc(&buf[i][j], cap[j]));
    slots = std::max(slots, want);
    return RS_OK;
  }
  int finish() {
    for (int i = 0; i < slots; i++) HIP_TRY(hipStreamSynchronize(st[i]));
    return RS_OK;
  }
};

// ring shape (env, read per call): RS_AMD_HOST_SLOTS (1..8, default 2) slices of
// RS_AMD_HOST_SLICE_MB input MiB (default 256). Pinned RS(10,4) 1 MiB x 512 encode /
// reconstruct GiB/s: 1 slot 37.5 / 37.0, 2 slots 49.3 / 49.8, 3 slots 44.6 / 48.8,
// 6 x 64 MiB 46.4 / 46.2 (profiles/r01/e2e_shapes): two slices keep one H2D, one
// kernel and one D2H in flight; more streams only contend for the copy engines.
int host_slots() {
  const char *e = std::getenv("RS_AMD_HOST_SLOTS");
  return e && *e ? std::max(1, std::min(Pipeline::kMaxSlots, std::atoi(e))) : 2;
}
// A slice's present shards cross PCIe as one strided copy per run of present rows; a run
// bridges gaps of up to RS_AMD_HOST_GAP missing rows (their bytes are copied too and never
// read: the caller's arrays hold every row); -1: one copy per row (round 5, measurement
// baseline). Measured: DESIGN.md §6 e2e.
int64_t host_gap_rows() {
  const char *e = std::getenv("RS_AMD_HOST_GAP");
  return e && *e ? std::max(-1, std::atoi(e)) : 0;
}
// [first, last) runs of present[0, rows) with gaps of <= gap missing rows bridged
std::vector<std::pair<uint64_t, uint64_t>> present_runs(const uint8_t *present, uint64_t rows, int64_t gap) {
  std::vector<std::pair<uint64_t, uint64_t>> runs;
  for (uint64_t j = 0; j < rows; j++) {
    if (!present[j]) continue;
    if (!runs.empty() && gap >= 0 && j - runs.back().second <= static_cast<uint64_t>(gap))
      runs.back().second = j + 1;
    else
      runs.emplace_back(j, j + 1);
  }
  return runs;
}
uint64_t host_slice_bytes() {
  const char *e = std::getenv("RS_AMD_HOST_SLICE_MB");
  return (e && *e ? static_cast<uint64_t>(std::max(1, std::atoi(e))) : 256ull) << 20;
}
// Stripes per reconstruct slice: the default 256 MiB, widened (up to 1 GiB) until the narrowest
// run's copy moves >= 8 MiB — c4 with every third data shard lost copies 2-row runs of 256 KiB
// shards: 46.7 / 48.9 / 49.3 GiB/s at 256 / 512 / 1024 MiB slices, where RS(10,4)'s 6-row runs of
// 1 MiB shards want 256 (50.0 / 49.3 / 47.8; profiles/r06/e2e/slice/). RS_AMD_HOST_SLICE_MB fixes it.
uint64_t reconstruct_slice_stripes(uint64_t n, uint64_t stripe_bytes, uint64_t sb,
                                   const std::vector<std::pair<uint64_t, uint64_t>> &runs) {
  uint64_t S = std::max<uint64_t>(1, host_slice_bytes() / stripe_bytes);
  const char *e = std::getenv("RS_AMD_HOST_SLICE_MB");
  if (!(e && *e)) {
    uint64_t narrow = UINT64_MAX;
    for (const auto &r : runs) narrow = std::min(narrow, (r.second - r.first) * sb);
    if (narrow != UINT64_MAX) {
      const uint64_t want = ((8ull << 20) + narrow - 1) / narrow;
      S = std::max(S, std::min(want, std::max<uint64_t>(1, (1ull << 30) / stripe_bytes)));
    }
  }
  return std::min(S, n);
}

// Fault injection for the error-path test (the reference's checkAllAllocationFailures,
// tests.zig:131-156, in spirit): RS_AMD_INJECT_HOST_FAIL=i fails slice i of a host batch.
bool inject_host_failure(uint64_t slice) {
  const char *e = std::getenv("RS_AMD_INJECT_HOST_FAIL");
  return e && *e && std::strtoull(e, nullptr, 10) == slice;
}

// process-lifetime rings (never freed: the HIP runtime reclaims them at exit)
std::mutex g_pipe_mu;
std::map<int, Pipeline *> g_pipes;

struct Pipelines {
  static Pipeline &of(int dev) {
    std::lock_guard<std::mutex> lk(g_pipe_mu);
    Pipeline *&p = g_pipes[dev];
    if (!p) p = new Pipeline();
    return *p;
  }
};

}  // namespace

void rs::host::release_host_rings() {
  std::lock_guard<std::mutex> lk(g_pipe_mu);
  for (auto &kv : g_pipes) {
    Pipeline &p = *kv.second;
    std::lock_guard<std::mutex> pk(p.mu);
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(kv.first);
    for (int i = 0; i < Pipeline::kMaxSlots; i++)
      for (int j = 0; j < 3; j++) {
        if (p.buf[i][j]) (void)hipFree(p.buf[i][j]);
        p.buf[i][j] = nullptr;
      }
    p.slots = 0;
    for (int j = 0; j < 3; j++) p.cap[j] = 0;
    for (int i = 0; i < Pipeline::kMaxSlots; i++)
      for (int j = 0; j < 3; j++) {
        if (p.hst[i][j]) (void)hipHostFree(p.hst[i][j]);
        p.hst[i][j] = nullptr;
      }
    p.hslots = 0;
    for (int j = 0; j < 3; j++) p.hcap[j] = 0;
    (void)hipSetDevice(cur);
  }
}

extern "C" {

int rs_encode_batch_host(uint64_t k, uint64_t m, size_t sb, uint64_t n, const void *h_orig, uint64_t orig_stride,
                         void *h_rec, uint64_t rec_stride, uint32_t flags) {
  TraceScope ts;
  return guarded([&]() -> int {
    if (k == 0) return fail(RS_ERR_TOO_FEW_ORIGINAL_SHARDS, "original_count == 0");
    int st = check_codec(k, m, sb);
    if (st) return st;
    if (n == 0) return RS_OK;
    if (!h_orig || !h_rec) return fail(RS_ERR_INVALID_ARGUMENT, "NULL host pointer");
    if (orig_stride == 0) orig_stride = k * sb;
    if (rec_stride == 0) rec_stride = m * sb;
    int dev;
    if ((st = current_device(&dev))) return st;
    const uint64_t S = std::max<uint64_t>(1, std::min<uint64_t>(n, host_slice_bytes() / (k * sb)));
    const int slots = host_slots();
    Pipeline &p = Pipelines::of(dev);
    std::lock_guard<std::mutex> lk(p.mu);
    const uint64_t bytes[3] = {S * k * sb, S * m * sb, 0};
    if ((st = p.ensure(bytes, slots))) return st;
    const bool stage = host_stage_on() && !(is_pinned(h_orig) && is_pinned(h_rec));
    if (stage && (st = p.ensure_stage(bytes, slots))) return st;
    uint64_t pend_s0[Pipeline::kMaxSlots] = {}, pend_cnt[Pipeline::kMaxSlots] = {};
    // staged: a slot's previous slice is waited for and its parity copied out before the slot's
    // staging buffers take the next slice
    auto take_out = [&](int slot) {
      if (!pend_cnt[slot]) return;
      host_copy({{static_cast<uint8_t *>(h_rec) + pend_s0[slot] * rec_stride, rec_stride,
                  static_cast<const uint8_t *>(p.hst[slot][1]), m * sb, m * sb, pend_cnt[slot]}});
      pend_cnt[slot] = 0;
    };
    auto slices = [&]() -> int {
      for (uint64_t s0 = 0, i = 0; s0 < n; s0 += S, i++) {
        const int slot = static_cast<int>(i % static_cast<uint64_t>(slots));
        const uint64_t cnt = std::min(S, n - s0);
        hipStream_t q = p.st[slot];
        if (inject_host_failure(i)) return fail(RS_ERR_DEVICE, "injected host-batch failure");
        const uint8_t *src = static_cast<const uint8_t *>(h_orig) + s0 * orig_stride;
        uint64_t src_stride = orig_stride;
        if (stage) {
          HIP_TRY(hipStreamSynchronize(q));
          take_out(slot);
          host_copy({{static_cast<uint8_t *>(p.hst[slot][0]), k * sb, src, orig_stride, k * sb, cnt}});
          src = static_cast<const uint8_t *>(p.hst[slot][0]);
          src_stride = k * sb;
        }
        HIP_TRY(copy_rows(p.buf[slot][0], k * sb, src, src_stride, k * sb, cnt, hipMemcpyHostToDevice, q));
        int rc = rs_encode_batch_dev(k, m, sb, cnt, p.buf[slot][0], 0, p.buf[slot][1], 0, flags, q);
        if (rc) return rc;
        if (stage) {
          HIP_TRY(copy_rows(p.hst[slot][1], m * sb, p.buf[slot][1], m * sb, m * sb, cnt, hipMemcpyDeviceToHost, q));
          pend_s0[slot] = s0;
          pend_cnt[slot] = cnt;
        } else {
          HIP_TRY(copy_rows(static_cast<uint8_t *>(h_rec) + s0 * rec_stride, rec_stride, p.buf[slot][1], m * sb,
                            m * sb, cnt, hipMemcpyDeviceToHost, q));
        }
      }
      return RS_OK;
    };
    // every slot stream is drained before the call returns, also after an error: no copy into
    // the caller's buffers (or out of them) outlives the call
    const int rc = slices(), fin = p.finish();
    if (stage && fin == RS_OK)
      for (int slot = 0; slot < slots; slot++) take_out(slot);  // slices that completed, also before an error
    return rc ? rc : fin;
  });
}

int rs_reconstruct_batch_host(uint64_t k, uint64_t m, size_t sb, uint64_t n, const uint8_t *present,
                              const void *h_orig, uint64_t orig_stride, const void *h_rec, uint64_t rec_stride,
                              void *h_out, uint64_t out_stride, uint32_t flags) {
  TraceScope ts;
  return guarded([&]() -> int {
    if (!present) return fail(RS_ERR_INVALID_ARGUMENT, "present == NULL");
    int st = check_codec(k, m, sb);
    if (st) return st;
    uint64_t e = 0, have = 0;
    for (uint64_t i = 0; i < k; i++) e += present[i] ? 0 : 1;
    for (uint64_t i = 0; i < k + m; i++) have += present[i] ? 1 : 0;
    if (have < k) return fail(RS_ERR_NOT_ENOUGH_SHARDS, "fewer than original_count shards present");
    if (e == 0 || n == 0) return RS_OK;
    if (!h_orig || !h_rec || !h_out) return fail(RS_ERR_INVALID_ARGUMENT, "NULL host pointer");
    if (orig_stride == 0) orig_stride = k * sb;
    if (rec_stride == 0) rec_stride = m * sb;
    if (out_stride == 0) out_stride = e * sb;
    int dev;
    if ((st = current_device(&dev))) return st;
    const int64_t gap = host_gap_rows();
    const auto runs_o = present_runs(present, k, gap), runs_r = present_runs(present + k, m, gap);
    auto runs_all = runs_o;
    runs_all.insert(runs_all.end(), runs_r.begin(), runs_r.end());
    const uint64_t S = reconstruct_slice_stripes(n, k * sb, sb, runs_all);
    const int slots = host_slots();
    Pipeline &p = Pipelines::of(dev);
    std::lock_guard<std::mutex> lk(p.mu);
    const uint64_t bytes[3] = {S * k * sb, S * m * sb, S * e * sb};
    if ((st = p.ensure(bytes, slots))) return st;
    const bool stage = host_stage_on() && !(is_pinned(h_orig) && is_pinned(h_rec) && is_pinned(h_out));
    if (stage && (st = p.ensure_stage(bytes, slots))) return st;
    uint64_t pend_s0[Pipeline::kMaxSlots] = {}, pend_cnt[Pipeline::kMaxSlots] = {};
    auto take_out = [&](int slot) {
      if (!pend_cnt[slot]) return;
      host_copy({{static_cast<uint8_t *>(h_out) + pend_s0[slot] * out_stride, out_stride,
                  static_cast<const uint8_t *>(p.hst[slot][2]), e * sb, e * sb, pend_cnt[slot]}});
      pend_cnt[slot] = 0;
    };
    auto slices = [&]() -> int {
      for (uint64_t s0 = 0, i = 0; s0 < n; s0 += S, i++) {
        const int slot = static_cast<int>(i % static_cast<uint64_t>(slots));
        const uint64_t cnt = std::min(S, n - s0);
        hipStream_t q = p.st[slot];
        if (inject_host_failure(i)) return fail(RS_ERR_DEVICE, "injected host-batch failure");
        const uint8_t *so = static_cast<const uint8_t *>(h_orig) + s0 * orig_stride;
        const uint8_t *sr = static_cast<const uint8_t *>(h_rec) + s0 * rec_stride;
        uint64_t sos = orig_stride, srs = rec_stride;
        if (stage) {  // the present rows into the slot's staging, in the device layout
          HIP_TRY(hipStreamSynchronize(q));
          take_out(slot);
          std::vector<CopyJob> jobs;
          uint8_t *ho = static_cast<uint8_t *>(p.hst[slot][0]), *hr = static_cast<uint8_t *>(p.hst[slot][1]);
          for (const auto &r : runs_o)
            jobs.push_back({ho + r.first * sb, k * sb, so + r.first * sb, orig_stride, (r.second - r.first) * sb, cnt});
          for (const auto &r : runs_r)
            jobs.push_back({hr + r.first * sb, m * sb, sr + r.first * sb, rec_stride, (r.second - r.first) * sb, cnt});
          host_copy(jobs);
          so = ho;
          sr = hr;
          sos = k * sb;
          srs = m * sb;
        }
        // only the present shards cross PCIe (and bridged gaps), one copy per run of rows
        for (const auto &r : runs_o)
          HIP_TRY(copy_rows(static_cast<uint8_t *>(p.buf[slot][0]) + r.first * sb, k * sb, so + r.first * sb, sos,
                            (r.second - r.first) * sb, cnt, hipMemcpyHostToDevice, q));
        for (const auto &r : runs_r)
          HIP_TRY(copy_rows(static_cast<uint8_t *>(p.buf[slot][1]) + r.first * sb, m * sb, sr + r.first * sb, srs,
                            (r.second - r.first) * sb, cnt, hipMemcpyHostToDevice, q));
        int rc = rs_reconstruct_batch_dev(k, m, sb, cnt, present, p.buf[slot][0], 0, p.buf[slot][1], 0,
                                          p.buf[slot][2], 0, flags, q);
        if (rc) return rc;
        if (stage) {
          HIP_TRY(copy_rows(p.hst[slot][2], e * sb, p.buf[slot][2], e * sb, e * sb, cnt, hipMemcpyDeviceToHost, q));
          pend_s0[slot] = s0;
          pend_cnt[slot] = cnt;
        } else {
          HIP_TRY(copy_rows(static_cast<uint8_t *>(h_out) + s0 * out_stride, out_stride, p.buf[slot][2], e * sb,
                            e * sb, cnt, hipMemcpyDeviceToHost, q));
        }
      }
      return RS_OK;
    };
    const int rc = slices(), fin = p.finish();
    if (stage && fin == RS_OK)
      for (int slot = 0; slot < slots; slot++) take_out(slot);
    return rc ? rc : fin;
  });
}

}  // extern "C"

namespace {
// One worker thread per device over contiguous stripe ranges (sharding.stripe_range's
// partition); each worker selects its device and calls the single-device host batch.
template <class F>
int run_multi(uint64_t n, const int *devices, int n_devices, F &&one) {
  std::vector<int> devs;
  if (devices) {
    if (n_devices <= 0) return fail(RS_ERR_INVALID_ARGUMENT, "n_devices <= 0");
    devs.assign(devices, devices + n_devices);
  } else {
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess || cnt <= 0) return fail(RS_ERR_NO_DEVICE, "no HIP device");
    for (int d = 0; d < cnt; d++) devs.push_back(d);
  }
  const uint64_t D = devs.size();
  std::vector<int> status(D, RS_OK);
  std::vector<std::string> msg(D);
  std::vector<std::thread> th;
  th.reserve(D);
  for (uint64_t i = 0; i < D; i++) {
    const uint64_t b = n * i / D, e = n * (i + 1) / D;
    th.emplace_back([&, i, b, e] {
      if (hipSetDevice(devs[i]) != hipSuccess) {
        status[i] = RS_ERR_NO_DEVICE;
        msg[i] = "hipSetDevice(" + std::to_string(devs[i]) + ") failed";
        return;
      }
      status[i] = e > b ? one(b, e - b) : RS_OK;
      if (status[i]) msg[i] = rs_last_error();
    });
  }
  for (auto &t : th) t.join();
  for (uint64_t i = 0; i < D; i++)
    if (status[i]) return fail(status[i], "device " + std::to_string(devs[i]) + ": " + msg[i]);
  return RS_OK;
}
}  // namespace

extern "C" {

int rs_encode_batch_host_multi(uint64_t k, uint64_t m, size_t sb, uint64_t n, const void *h_orig, uint64_t orig_stride,
                               void *h_rec, uint64_t rec_stride, uint32_t flags, const int *devices, int n_devices) {
  TraceScope ts;
  return guarded([&]() -> int {
    if (orig_stride == 0) orig_stride = k * sb;
    if (rec_stride == 0) rec_stride = m * sb;
    return run_multi(n, devices, n_devices, [&](uint64_t s0, uint64_t cnt) {
      return rs_encode_batch_host(k, m, sb, cnt, static_cast<const uint8_t *>(h_orig) + s0 * orig_stride,
                                  orig_stride, static_cast<uint8_t *>(h_rec) + s0 * rec_stride, rec_stride, flags);
    });
  });
}

int rs_reconstruct_batch_host_multi(uint64_t k, uint64_t m, size_t sb, uint64_t n, const uint8_t *present,
                                    const void *h_orig, uint64_t orig_stride, const void *h_rec, uint64_t rec_stride,
                                    void *h_out, uint64_t out_stride, uint32_t flags, const int *devices,
                                    int n_devices) {
  TraceScope ts;
  return guarded([&]() -> int {
    if (!present) return fail(RS_ERR_INVALID_ARGUMENT, "present == NULL");
    uint64_t e = 0;
    for (uint64_t i = 0; i < k; i++) e += present[i] ? 0 : 1;
    if (orig_stride == 0) orig_stride = k * sb;
    if (rec_stride == 0) rec_stride = m * sb;
    if (out_stride == 0) out_stride = e * sb;
    return run_multi(n, devices, n_devices, [&](uint64_t s0, uint64_t cnt) {
      return rs_reconstruct_batch_host(k, m, sb, cnt, present, static_cast<const uint8_t *>(h_orig) + s0 * orig_stride,
                                       orig_stride, static_cast<const uint8_t *>(h_rec) + s0 * rec_stride, rec_stride,
                                       static_cast<uint8_t *>(h_out) + s0 * out_stride, out_stride, flags);
    });
  });
}

}  // extern "C"
