// rs_common.cpp — errors, device checks, validation (root.zig:397-415 and the
// Encoder/Decoder init checks), plan-cache plumbing, kernel slots, and the info ABI.
#include "rs_host.hpp"

namespace rs {
namespace host {

thread_local std::string t_last_error;

int fail(int status, const std::string &msg) {
  t_last_error = msg;
  return status;
}

int hip_fail(hipError_t e, const char *what) {
  // the failed call also set the thread's last HIP error: reset it, so the caller's next
  // hipGetLastError (e.g. torch's launch check) does not report this call's failure
  (void)hipGetLastError();
  return fail(e == hipErrorOutOfMemory ? RS_ERR_OUT_OF_MEMORY : RS_ERR_DEVICE,
              std::string(what) + ": " + hipGetErrorString(e));
}

// ------------------------------------------------------ allocation-failure injection
namespace {
std::atomic<int64_t> g_fail_at{-1};  // index of the allocation that fails (-1: off)
std::atomic<int64_t> g_allocs{0};    // allocations counted since rs_debug_fail_alloc
}  // namespace

bool alloc_fails() {
  const int64_t i = g_allocs.fetch_add(1);
  return i == g_fail_at.load();
}

void alloc_point() {
  if (alloc_fails()) throw std::bad_alloc();
}

hipError_t dev_malloc(void **p, size_t bytes) {
  if (alloc_fails()) {
    *p = nullptr;
    return hipErrorOutOfMemory;
  }
  return hipMalloc(p, bytes);
}

hipError_t dev_malloc_async(void **p, size_t bytes, hipStream_t s) {
  if (alloc_fails()) {
    *p = nullptr;
    return hipErrorOutOfMemory;
  }
  return hipMallocAsync(p, bytes, s);
}

hipError_t pinned_malloc(void **p, size_t bytes) {
  if (alloc_fails()) {
    *p = nullptr;
    return hipErrorOutOfMemory;
  }
  return hipHostMalloc(p, bytes, hipHostMallocDefault);
}

int64_t arm_alloc_failure(int64_t n) {
  const int64_t seen = g_allocs.exchange(0);
  g_fail_at.store(n < 0 ? -1 : n);
  return seen;
}


const char *last_error() { return t_last_error.c_str(); }

}  // namespace host

// ---------------------------------------------------------- launch record
namespace {
thread_local std::string t_trace;       // names joined by ';' in launch order
thread_local std::string t_trace_last;  // collapse repeats (slices of one batch)
thread_local int t_trace_depth = 0;
}  // namespace

void trace_launch(const char *name) {
  if (!name || t_trace_last == name) return;
  t_trace_last = name;
  if (!t_trace.empty()) t_trace.push_back(';');
  t_trace += name;
}

TraceScope::TraceScope() {
  if (t_trace_depth++ == 0) {
    t_trace.clear();
    t_trace_last.clear();
  }
}
TraceScope::~TraceScope() { t_trace_depth--; }

const char *trace_text() { return t_trace.c_str(); }

namespace host {

// ---------------------------------------------------------------- devices
std::mutex g_dev_mu;
std::map<int, int> g_dev_ok;  // device -> RS_OK / RS_ERR_NO_DEVICE

namespace {
std::atomic<bool> g_process_exiting{false};
void mark_process_exiting() { g_process_exiting.store(true); }
}  // namespace
bool process_exiting() { return g_process_exiting.load(); }

int current_device(int *dev) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(RS_ERR_NO_DEVICE, "no HIP device visible");
  HIP_TRY(hipGetDevice(dev));
  static std::once_flag exit_once;  // after the runtime's initialisation: runs before its teardown
  std::call_once(exit_once, [] { std::atexit(mark_process_exiting); });
  std::lock_guard<std::mutex> lk(g_dev_mu);
  auto it = g_dev_ok.find(*dev);
  if (it == g_dev_ok.end()) {
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, *dev));
    const bool ok = std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
    it = g_dev_ok.emplace(*dev, ok ? RS_OK : RS_ERR_NO_DEVICE).first;
    if (!ok) return fail(RS_ERR_NO_DEVICE, std::string("device arch ") + prop.gcnArchName + " is not gfx950");
  }
  if (it->second != RS_OK) return fail(it->second, "device is not gfx950");
  return RS_OK;
}

// ------------------------------------------------------------ validation
// root.zig:397-415
int use_high_rate(uint64_t original, uint64_t recovery) {
  if (original > kOrder || recovery > kOrder) return -RS_ERR_UNSUPPORTED_SHARD_COUNT;
  if (original == 0 || recovery == 0) return -RS_ERR_UNSUPPORTED_SHARD_COUNT;  // ceilPowerOfTwo(0) asserts
  const uint64_t op = ceil_pow2(original), rp = ceil_pow2(recovery);
  const uint64_t smaller = std::min(op, rp), larger = std::max(original, recovery);
  if (smaller + larger > kOrder) return -RS_ERR_UNSUPPORTED_SHARD_COUNT;
  if (op < rp) return 0;
  if (op > rp) return 1;
  return original <= recovery ? 1 : 0;
}

// Encoder.init / Decoder.init checks (root.zig:100-103, 198-201) + the tail panic (root.zig:385)
int check_codec(uint64_t k, uint64_t m, size_t shard_bytes) {
  const int hr = use_high_rate(k, m);
  if (hr < 0) return fail(-hr, "unsupported shard count (root.zig:397-415)");
  // low rate (hr == 0): the reference panics (root.zig:120, 227); here rs_lowrate.cpp (§8 f4)
  if (shard_bytes == 0 || (shard_bytes & 1)) return fail(RS_ERR_INVALID_SHARD_SIZE, "shard_bytes is 0 or odd");
  // shard_bytes % 64 != 0: the reference panics (root.zig:385); handled here with
  // the tail layout of root.zig:338-348 (tail_* below).
  return RS_OK;
}

int align_nv(std::initializer_list<uint64_t> vals) {
  uint64_t a = 0;
  for (uint64_t v : vals) a |= v;
  if (a % 16 == 0) return 4;
  if (a % 8 == 0) return 2;
  if (a % 4 == 0) return 1;
  return 0;
}

uint32_t async_after() {
  const char *e = std::getenv("RS_AMD_NET_ASYNC_AFTER");
  return e && *e ? static_cast<uint32_t>(std::max(1, std::atoi(e))) : 2u;
}

// A fallback to the table kernels is reported on stderr once per distinct reason.
void warn_once_per_reason(const char *what, const std::string &err) {
  static std::mutex mu;
  static std::set<std::string> seen;
  std::lock_guard<std::mutex> lk(mu);
  if (seen.insert(err.substr(0, 200)).second) std::fprintf(stderr, "%s%s\n", what, err.c_str());
}

bool fft_enabled() {
  const char *e = std::getenv("RS_AMD_FFT");
  return jit::enabled() && !(e && std::strcmp(e, "0") == 0);
}

// The slot's kernel for shards of sb bytes; *used = the spec to launch it with.
const jit::Kernel *fft_kernel(FftSlot &slot, uint64_t sb, const fftnet::Spec **used) {
  std::lock_guard<std::mutex> lk(slot.mu);
  const int vi = fftnet::pieces(sb) > 1 ? 1 : 0;
  if (slot.failed[vi]) return nullptr;
  if (vi && slot.spec_p2.pieces == 1) {
    slot.spec_p2 = slot.spec;
    slot.spec_p2.pieces = 2;
  }
  const fftnet::Spec &spec = vi ? slot.spec_p2 : slot.spec;
  *used = &spec;
  std::string err;
  bool pending = false;
  const bool async = slot.async;
  const jit::Kernel *k = fftnet::get(spec, async, err, pending);
  if (!k && !pending) {
    slot.failed[vi] = true;
    warn_once_per_reason("[rs_amd] bit-sliced FFT kernel unavailable, using table kernels: ", err);
  }
  return k;
}

// Compile (once) and return the plan's network kernel; nullptr if hipRTC failed
// (the caller then runs the precompiled table-driven kernels).
// (jit::get caches by content and code-shape knobs; a failure is reported once per plan.)
// An async slot returns nullptr (table kernels) until its background compile is done.
// 1 / 2 KiB shards run a variant whose wave units span 4 / 2 stripes (jit::net_pieces).
const jit::Kernel *net_kernel(NetSlot &slot, uint64_t sb) {
  std::lock_guard<std::mutex> lk(slot.mu);
  const uint32_t pieces = jit::net_pieces(sb);
  const int vi = pieces >= 4 ? 2 : pieces >= 2 ? 1 : 0;  // a failed variant does not disable the others
  if (slot.failed[vi]) return nullptr;
  std::string err;
  bool pending = false;
  if (slot.async && slot.uses < async_after()) {  // a one-off pattern is not worth a background compile
    const char *sync = std::getenv("RS_AMD_JIT_SYNC");
    if (!(sync && *sync && std::strcmp(sync, "0") != 0) && ++slot.uses < async_after()) return nullptr;
  }
  jit::NetSpec small;
  if (pieces > 1) {
    small = slot.spec;
    small.pieces = pieces;
  }
  const jit::NetSpec &spec = pieces > 1 ? small : slot.spec;
  const jit::Kernel *k = slot.async ? jit::get_async(spec, err, pending) : jit::get(spec, err);
  if (!k && !pending) {
    slot.failed[vi] = true;
    warn_once_per_reason("[rs_amd] bit-sliced network unavailable, using table kernels: ", err);
  }
  return k;
}

void queue_net(NetSlot &slot, uint64_t sb) {
  {
    std::lock_guard<std::mutex> lk(slot.mu);
    slot.uses = std::max(slot.uses, async_after());  // a warmed pattern is not a one-off
  }
  (void)net_kernel(slot, sb);
}

std::mutex g_plan_mu;

namespace {
std::map<std::string, std::shared_ptr<DevBuf>> g_twiddle_plans;  // IFFT+FFT tables of size W, skew_delta 0
}  // namespace

int twiddle_plan(int dev, uint64_t W, uint32_t flags, std::shared_ptr<DevBuf> &out, size_t &off_fft) {
  const bool d1 = flags & RS_FLAG_QUIRK_D1;
  off_fft = ifft_tab_count(W) * sizeof(RsTab);
  const std::string key = std::to_string(dev) + "/" + std::to_string(W) + "/" + std::to_string(d1);
  {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    auto it = g_twiddle_plans.find(key);
    if (it != g_twiddle_plans.end()) {
      out = it->second;
      return RS_OK;
    }
  }
  std::vector<RsTab> tabs;  // built without the lock (65536-point tables take milliseconds)
  push_ifft_tabs(tabs, W, 0, d1);
  push_fft_tabs(tabs, W, 0, d1);
  std::shared_ptr<DevBuf> buf;
  if (int st = upload(tabs.data(), tabs.size() * sizeof(RsTab), dev, buf)) return st;
  std::lock_guard<std::mutex> lk(g_plan_mu);
  out = g_twiddle_plans.emplace(key, buf).first->second;  // first insert wins
  return RS_OK;
}

// Plan uploads go through private non-blocking streams: a synchronous hipMemcpy runs on the
// null stream, which orders itself against every blocking stream of the device — an upload
// from the background worker (a plan upgrade) would then wait for the caller's in-flight
// batches and delay its next launches. A small fixed pool per device (created once, each
// stream used under its own lock; ADVICE r4: one stream per thread leaked a stream per
// short-lived thread). The streams are never destroyed: a destructor at exit could run after
// the HIP runtime's teardown.
namespace {
constexpr int kUploadStreams = 4;
struct UploadPool {
  hipStream_t st[kUploadStreams] = {};
  std::mutex mu[kUploadStreams];
  std::atomic<uint32_t> next{0};
};
std::mutex g_upload_mu;
std::map<int, UploadPool *> g_upload_pools;  // never freed (see above)
}  // namespace

int upload(const void *host, size_t bytes, int dev, std::shared_ptr<DevBuf> &out) {
  UploadPool *pool = nullptr;
  {
    std::lock_guard<std::mutex> lk(g_upload_mu);
    UploadPool *&p = g_upload_pools[dev];
    if (!p) p = new UploadPool;
    pool = p;
  }
  auto b = std::make_shared<DevBuf>();
  b->dev = dev;
  HIP_TRY(dev_malloc(&b->p, std::max<size_t>(bytes, 16)));
  const uint32_t i = pool->next.fetch_add(1) % kUploadStreams;
  std::lock_guard<std::mutex> lk(pool->mu[i]);
  if (!pool->st[i]) HIP_TRY(hipStreamCreateWithFlags(&pool->st[i], hipStreamNonBlocking));
  HIP_TRY(hipMemcpyAsync(b->p, host, bytes, hipMemcpyHostToDevice, pool->st[i]));
  HIP_TRY(hipStreamSynchronize(pool->st[i]));
  out = b;
  return RS_OK;
}

}  // namespace host
}  // namespace rs

using namespace rs;
using namespace rs::host;

extern "C" {

const char *rs_version(void) { return "rs-amd 0.1.0 (gfx950)"; }

const char *rs_status_name(int s) {
  static const char *kNames[] = {"Ok",
                                 "TooFewOriginalShards",
                                 "NotEnoughShards",
                                 "InvalidShardSize",
                                 "UnsupportedShardCount",
                                 "TooManyOriginalShards",
                                 "DifferentShardSize",
                                 "InvalidShardIndex",
                                 "DuplicateShardIndex",
                                 "TooManyShards",
                                 "OutOfMemory",
                                 "Overflow",
                                 "LowRateUnsupported",
                                 "ShardTailUnsupported",
                                 "InvalidArgument",
                                 "DeviceError",
                                 "NoDevice"};
  if (s < 0 || s >= static_cast<int>(sizeof kNames / sizeof kNames[0])) return "Unknown";
  return kNames[s];
}

const char *rs_last_error(void) { return last_error(); }

const char *rs_last_kernels(void) { return trace_text(); }

int rs_use_high_rate(uint64_t k, uint64_t m) { return use_high_rate(k, m); }

const uint16_t *rs_table_exp(void) { return tables().exp; }
const uint16_t *rs_table_log(void) { return tables().log; }
const uint16_t *rs_table_skew(void) { return tables().skew; }
const uint16_t *rs_table_log_walsh(void) { return tables().log_walsh; }
const uint8_t *rs_table_mul_128(void) {  // tables.zig:94-118
  static const uint8_t *t = []() -> const uint8_t * {
    uint8_t *p = static_cast<uint8_t *>(std::malloc(size_t(kOrder) * 128));
    if (!p) return nullptr;
    for (uint32_t lm = 0; lm < kOrder; lm++)
      for (uint32_t i = 0; i < 4; i++)
        for (uint32_t j = 0; j < 16; j++) {
          const uint16_t prod = mul16(static_cast<uint16_t>(j << (4 * i)), static_cast<uint16_t>(lm));
          p[size_t(lm) * 128 + i * 16 + j] = static_cast<uint8_t>(prod);
          p[size_t(lm) * 128 + 64 + i * 16 + j] = static_cast<uint8_t>(prod >> 8);
        }
    return p;
  }();
  return t;
}

int rs_jit_stats(uint64_t *compiles, uint64_t *cache_hits, uint64_t *modules) {
  return guarded([&]() -> int {
    jit::compile_stats(compiles, cache_hits, modules);
    return RS_OK;
  });
}

// The counter is process-wide: a plan upgrade or compile still queued from an earlier call
// would otherwise take the armed index on the background worker, so the worker
// is drained before arming.
int64_t rs_debug_fail_alloc(int64_t n) {
  jit::wait_pending();
  return arm_alloc_failure(n);
}

int rs_debug_release_caches(uint64_t *pooled_contexts) {
  return guarded([&]() -> int {
    jit::wait_pending();  // no plan build on the worker holds a plan being dropped
    release_plans();
    release_patterns();
    release_lowrate();
    release_oneshot();
    release_host_rings();
    {
      std::lock_guard<std::mutex> lk(g_plan_mu);
      g_twiddle_plans.clear();
    }
    if (pooled_contexts) *pooled_contexts = oneshot_pooled();
    return RS_OK;
  });
}

int64_t rs_debug_erasure_logs_check(uint64_t k, uint64_t m, const uint8_t *received, int low) {
  if (!received || k == 0 || m == 0 || k + m > kOrder) return -1;
  const uint64_t C = ceil_pow2(low ? k : m), end = C + (low ? m : k), W = ceil_pow2(end);
  if (W > kOrder) return -1;
  std::vector<uint16_t> a(kOrder), b(kOrder);
  std::vector<uint8_t> rcv(received, received + end);
  rcv.resize(W, 0);
  set_erasure_logs_fwht(false);
  (low ? erasure_logs_low : erasure_logs)(rcv.data(), k, m, a.data());
  set_erasure_logs_fwht(true);
  (low ? erasure_logs_low : erasure_logs)(rcv.data(), k, m, b.data());
  set_erasure_logs_fwht(false);
  int64_t bad = 0;
  for (uint64_t i = 0; i < W; i++) bad += a[i] % kModulus != b[i] % kModulus;
  return bad;
}

int rs_net_wait(void) {
  return guarded([&]() -> int {
    jit::wait_pending();
    return RS_OK;
  });
}

}  // extern "C"
