// rs_host.hpp — internal interface of the host codec (librs_amd.so): validation and
// error reporting, plan caches, kernel selection, plans, and the entry points the
// C ABI files (rs_batch_dev.cpp, rs_patterns.cpp, rs_lowrate.cpp, rs_host_batch.cpp,
// rs_oneshot.cpp) share. Host-side mirror of root.zig's checks and error
// precedence; every device computation runs in rs_kernels.hip or in a hipRTC
// kernel (rs_jit / rs_fftnet / rs_psyn); there is no CPU compute path.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/reedsol.h"
#include "rs_fftnet.hpp"
#include "rs_gf.hpp"
#include "rs_internal.hpp"
#include "rs_jit.hpp"
#include "rs_psyn.hpp"

namespace rs {
namespace host {

// ------------------------------------------------------------ errors (rs_common.cpp)
int fail(int status, const std::string &msg);  // sets rs_last_error()
int hip_fail(hipError_t e, const char *what);   // hipErrorOutOfMemory -> RS_ERR_OUT_OF_MEMORY
const char *last_error();

// Allocation-failure injection (rs_debug_fail_alloc; the reference's
// checkAllAllocationFailures, tests.zig:131-156): every allocation the library makes
// — plan objects (alloc_point, throws std::bad_alloc), device, async-pool and pinned
// buffers (the wrappers, hipErrorOutOfMemory) — is counted, and the armed one fails.
bool alloc_fails();
void alloc_point();
hipError_t dev_malloc(void **p, size_t bytes);
hipError_t dev_malloc_async(void **p, size_t bytes, hipStream_t s);
hipError_t pinned_malloc(void **p, size_t bytes);
int64_t arm_alloc_failure(int64_t n);  // returns the allocations counted since the last call
// Drop every cache that holds device or pinned memory (plans, tables, staging rings,
// one-shot contexts); compiled kernels stay loaded (rs_debug_release_caches).
void release_plans();      // rs_plans.cpp (+ twiddles, rs_common.cpp)
void release_patterns();   // rs_patterns.cpp
void release_lowrate();    // rs_lowrate.cpp
void release_oneshot();    // rs_oneshot.cpp
size_t oneshot_pooled();   // one-shot contexts idle in the pool
void release_host_rings(); // rs_host_batch.cpp

#define HIP_TRY(expr)                               \
  do {                                              \
    hipError_t e_ = (expr);                         \
    if (e_ != hipSuccess) return hip_fail(e_, #expr); \
  } while (0)

// No C++ exception may cross the C ABI: host allocation failures become
// RS_ERR_OUT_OF_MEMORY, anything else RS_ERR_DEVICE with its message.
template <class F>
int guarded(F &&f) {
  try {
    return f();
  } catch (const std::bad_alloc &) {
    return fail(RS_ERR_OUT_OF_MEMORY, "host allocation failed");
  } catch (const std::exception &ex) {
    return fail(RS_ERR_DEVICE, ex.what());
  } catch (...) {
    return fail(RS_ERR_DEVICE, "unexpected exception");
  }
}

// ---------------------------------------------------- validation (rs_common.cpp)
int current_device(int *dev);  // RS_ERR_NO_DEVICE unless the current device is gfx950
// root.zig:397-415: 1 high rate, 0 low rate, -status on invalid counts
int use_high_rate(uint64_t original, uint64_t recovery);
inline bool is_low_rate(uint64_t k, uint64_t m) { return use_high_rate(k, m) == 0; }
// The reconstruct as written reads every present shard and is no decoder of the parity the
// encode wrote: under D1 (Generic.zig:283, the multiply) and under D2 when it drops a chunk
// (root.zig:151, k > chunk and k % chunk == 0: the parity ignores those shards). Such
// reconstructs run on maps of all present shards (no trimming to k inputs, no syndromes,
// no solve), so they stay bit-exact with the reference on any set of present shards.
inline bool literal_decode(uint64_t k, uint64_t m, uint32_t flags) {
  const uint64_t C = ceil_pow2(m);
  return (flags & RS_FLAG_QUIRK_D1) || ((flags & RS_FLAG_QUIRK_D2) && k > C && k % C == 0);
}
// Encoder.init / Decoder.init checks (root.zig:100-103, 198-201)
int check_codec(uint64_t k, uint64_t m, size_t shard_bytes);
// widest per-lane access (4, 2, 1 dword pairs) the alignment of every value allows; 0 = none
int align_nv(std::initializer_list<uint64_t> vals);

// ------------------------------------------------------- plans (rs_common.cpp)
// Set by an exit handler registered after the HIP runtime's (so it runs before the runtime's
// teardown): the plan caches' static destruction then skips HIP calls (the process is ending;
// freeing into a torn-down runtime can fault)
bool process_exiting();
struct DevBuf {
  void *p = nullptr;
  int dev = 0;
  ~DevBuf() {
    if (p && !process_exiting()) {
      int cur = 0;
      (void)hipGetDevice(&cur);
      (void)hipSetDevice(dev);
      (void)hipFree(p);
      (void)hipSetDevice(cur);
    }
  }
};

// Bit-sliced network kernel of a plan (rs_jit.hpp), compiled on first use.
struct NetSlot {
  std::mutex mu;
  bool failed[3] = {false, false, false};  // per variant: 4 KiB units, 2 / 4 stripes per unit (small shards)
  bool async = false;  // past the synchronous size cap: compiled in the background
  uint32_t uses = 0;   // async: the compile starts at the RS_AMD_NET_ASYNC_AFTER-th use (default 2)
  jit::NetSpec spec;
};

uint32_t async_after();  // RS_AMD_NET_ASYNC_AFTER
// A fallback to the table kernels is reported on stderr once per distinct reason.
void warn_once_per_reason(const char *what, const std::string &err);

// Bit-sliced FFT kernel of a plan (rs_fftnet.hpp): wide codes, compiled on first use.
struct FftSlot {
  std::mutex mu;
  bool failed[2] = {false, false};  // per variant: 2 KiB units of one stripe / of two 1 KiB stripes
  bool async = false;  // per-pattern kernels: background compile, the table encode meanwhile
  fftnet::Spec spec;
  fftnet::Spec spec_p2;  // the 1 KiB-shard variant (Spec::pieces 2), filled on first use
};

bool fft_enabled();
// The slot's kernel for shards of sb bytes; *used = the spec to launch it with.
const jit::Kernel *fft_kernel(FftSlot &slot, uint64_t sb, const fftnet::Spec **used);
// The slot's network kernel (compiled on first use; nullptr: table kernels)
const jit::Kernel *net_kernel(NetSlot &slot, uint64_t sb);
// Start the slot's compile now (an async slot: queued on the background worker, whatever
// its use count), e.g. when a plan upgrade or rs_reconstruct_warm knows it will be used.
void queue_net(NetSlot &slot, uint64_t sb);

struct EncodePlan {
  std::shared_ptr<DevBuf> buf;
  uint32_t chunk, n_chunks, trunc_first, trunc_last, tabs_per_chunk, work;
  std::shared_ptr<NetSlot> net = std::make_shared<NetSlot>();
  std::shared_ptr<FftSlot> fft;  // wide codes (chunk 32 / 64)
};

struct DecodePlan {
  std::shared_ptr<DevBuf> buf;
  bool matrix = false;
  bool tiled = false;
  uint32_t work = 0, chunk = 0, trunc = 0, e = 0, n_in = 0;
  size_t off_fft = 0, off_pre = 0, off_post = 0, off_src = 0, off_dst = 0, off_mat = 0;  // byte offsets into buf
  std::shared_ptr<NetSlot> net;  // set when the pattern runs as a bit-sliced network
  // reconstruct by syndromes: encode the received data (erased shards skipped) into
  // a scratch, then the e x e matrix kernel on rec ^ scratch rows (see syndrome_map)
  bool syndrome = false;
  std::shared_ptr<DevBuf> skip;  // k-bit mask of the erased data shards
  std::shared_ptr<FftSlot> inv_fft;  // every original lost, k == m == chunk: the encode inverted
  // the syndrome path on wide codes (chunk 32 / 64, whole 4 KiB units): the code's FFT
  // kernel with per-stripe masks (fftnet::Spec::dyn, compiled once per code) and, while
  // the pattern's e x e network compiles, the generic solve (rs_psyn.hpp) — one plan block
  // for the batch (fftnet masks, then at word syn_dmw the solve header and A^-1 in
  // polynomial form)
  std::shared_ptr<DevBuf> syn_blk;
  uint32_t syn_dmw = 0, syn_pw = 0, syn_cs = 0;
  // the fused FFT reconstruct (fftnet::Spec::decode): the pattern's
  // decode block (rows R, locator masks, output rows); the kernel is per code
  std::shared_ptr<DevBuf> fdec_blk;
  uint32_t fdec_words = 0;
  // the same reconstruct with this pattern compiled in (fftnet::Spec::present; background
  // compile): the steady state of a wide-code pattern unless a direct network beats it
  std::shared_ptr<FftSlot> pdec;
  // a pattern's first use builds only the fused block (no network spec, no tables: the
  // host GF(2) algebra of those takes 10-40 ms); where a network would beat the fused
  // kernel, its next use has the full plan built on the background worker
  bool lite = false;
  std::atomic<bool> upgrading{false};
  std::atomic<uint32_t> uses{1};  // calls that found this (lite) plan, the first included
};

// Plan caches: least-recently-used entries past RS_AMD_PLAN_CACHE (default 4096 per
// kind) are dropped (a plan in use stays alive through its shared_ptr). g_plan_mu
// guards the maps only: plans are built without it (double-checked insertion; two
// threads racing on a new key may both build, the first insert wins).
inline size_t plan_cache_cap() {
  const char *e = std::getenv("RS_AMD_PLAN_CACHE");
  return e && *e ? static_cast<size_t>(std::max(1, std::atoi(e))) : 4096u;
}

template <class V>
struct PlanCache {
  std::map<std::string, std::pair<std::shared_ptr<V>, uint64_t>> m;  // plan, last use
  uint64_t tick = 0;
  std::shared_ptr<V> find(const std::string &k) {  // g_plan_mu held
    auto it = m.find(k);
    if (it == m.end()) return nullptr;
    it->second.second = ++tick;
    return it->second.first;
  }
  std::shared_ptr<V> insert(const std::string &k, std::shared_ptr<V> v) {  // g_plan_mu held
    auto it = m.find(k);
    if (it != m.end()) {
      it->second.second = ++tick;
      return it->second.first;
    }
    const size_t cap = plan_cache_cap();
    if (m.size() >= cap) {  // drop the oldest eighth (amortised O(1) per insert)
      std::vector<std::pair<uint64_t, std::string>> age;
      age.reserve(m.size());
      for (auto &kv : m) age.emplace_back(kv.second.second, kv.first);
      const size_t drop = std::max<size_t>(1, m.size() - cap + cap / 8);
      std::nth_element(age.begin(), age.begin() + (drop - 1), age.end());
      for (size_t i = 0; i < drop; i++) m.erase(age[i].second);
    }
    m.emplace(k, std::make_pair(v, ++tick));
    return v;
  }
  std::shared_ptr<V> replace(const std::string &k, std::shared_ptr<V> v) {  // g_plan_mu held
    auto it = m.find(k);
    if (it == m.end()) return insert(k, v);
    it->second = std::make_pair(v, ++tick);
    return v;
  }
  size_t size() const { return m.size(); }
  void clear() { m.clear(); }  // g_plan_mu held
};

extern std::mutex g_plan_mu;
int upload(const void *host, size_t bytes, int dev, std::shared_ptr<DevBuf> &out);
// IFFT + FFT tables of size W at skew 0 (decode transforms), per (device, W, D1), in
// HBM for the life of the process; *off_fft = byte offset of the FFT tables
int twiddle_plan(int dev, uint64_t W, uint32_t flags, std::shared_ptr<DevBuf> &out, size_t &off_fft);

constexpr uint64_t kScratchCap = 2ull << 30;  // generic path: scratch per launch
// the generic kernels' scratch cap per launch: kScratchCap, or RS_AMD_SCRATCH_CAP_MB
inline uint64_t scratch_cap() {
  const char *e = std::getenv("RS_AMD_SCRATCH_CAP_MB");
  return e && *e ? std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) << 20 : kScratchCap;
}
// stripes per scratch slice: as many as fit the cap, spread evenly over the slices (a short
// last slice runs its launches at lower occupancy)
inline uint64_t slice_stripes(uint64_t n, uint64_t per_stripe_bytes) {
  const uint64_t fit = std::max<uint64_t>(1, std::min<uint64_t>(n, scratch_cap() / per_stripe_bytes));
  const uint64_t slices = (n + fit - 1) / fit;
  return (n + slices - 1) / slices;
}

// ------------------------------------------------- kernel selection (rs_select.cpp)
bool encode_net_async(uint64_t k, uint64_t m);
bool encode_net_ok(uint64_t sb);
uint64_t fft_decode_mul_count(uint64_t k, uint64_t m, uint64_t present_count, uint64_t e);
uint64_t fft_encode_mul_count(uint64_t k, uint64_t m);
const char *decode_mode_env();
constexpr uint32_t flags_none() { return 0; }
int decode_kind(uint64_t k, uint64_t m, uint32_t flags, uint64_t e, uint64_t present_count, uint64_t sb);
bool syndrome_pick(uint64_t k, uint64_t m, uint64_t e, uint32_t flags, uint64_t sb, const std::string &mode);
bool direct_net_async(uint64_t e, uint64_t n_in, uint64_t sb, const std::string &mode, uint64_t k, uint64_t m,
                      uint32_t flags);
const char *net_name(const char *role, uint64_t n_in, uint64_t n_out);

// ------------------------------------------------------------- plans (rs_plans.cpp)
void encode_map(uint64_t k, uint64_t m, uint32_t flags, jit::NetSpec &ns);
void reconstruct_map(uint64_t k, uint64_t m, uint32_t flags, const uint8_t *present, jit::NetSpec &ns);
int syndrome_map(uint64_t k, uint64_t m, const uint8_t *present, jit::NetSpec &ns);
int get_encode_plan(int dev, uint64_t k, uint64_t m, uint32_t flags, std::shared_ptr<EncodePlan> &out);
// how: 0 the cached plan (a lite plan schedules its upgrade when a network or the
// pattern-compiled kernel would win; counts a use), 1 never a lite plan (the fused kernel is
// unavailable), 2 build the full plan now (the background upgrade), 3 as 0 without counting
// a use and without the reuse / worker-backlog bounds (rs_reconstruct_warm)
int get_decode_plan(int dev, uint64_t k, uint64_t m, uint64_t sb, uint32_t flags, const uint8_t *present,
                    std::shared_ptr<DecodePlan> &out, int how = 0);

// ------------------------------------------------------ shard tails (rs_batch_dev.cpp)
// Batches whose shard_bytes is not a multiple of 64 run on padded copies
// ([stripe][shard][ceil(sb/64)*64], the tail chunk in the layout root.zig:338-348 implies)
// in slices of <= kTailSliceBytes.
constexpr uint64_t kTailSliceBytes = 1ull << 30;
int pad_shards(const uint8_t *src, uint64_t src_stripe_stride, uint64_t sb, uint8_t *dst, uint64_t dst_stripe_stride,
               uint64_t psb, uint64_t n, hipStream_t s);
int unpad_shards(const uint8_t *src, uint64_t src_stripe_stride, uint64_t sb, uint8_t *dst, uint64_t dst_stripe_stride,
                 uint64_t n, hipStream_t s);

// ---------------------------------------------------------- low rate (rs_lowrate.cpp)
int low_encode(int dev, uint64_t k, uint64_t m, uint64_t sb, uint64_t n, const uint8_t *orig, uint64_t ostride,
               uint8_t *rec, uint64_t rstride, uint32_t flags, int max_nv, hipStream_t s);
int low_reconstruct(int dev, uint64_t k, uint64_t m, uint64_t sb, uint64_t n, const uint8_t *present,
                    const uint8_t *orig, uint64_t ostride, const uint8_t *rec, uint64_t rstride, uint8_t *out,
                    uint64_t outstride, uint32_t flags, int max_nv, hipStream_t s);
// rs_reconstruct_warm for a low-rate pattern: its plan, and its network compiled
int low_warm(int dev, uint64_t k, uint64_t m, uint64_t sb, const uint8_t *present);
const char *low_encode_kernel_name(uint64_t k, uint64_t m, uint64_t sb);
const char *low_reconstruct_kernel_name(uint64_t k, uint64_t m, uint64_t sb, uint64_t e);
int low_decode_map(uint64_t k, uint64_t m, uint32_t flags, const uint8_t *present, jit::NetSpec &ns);
// the low-rate reconstruct in block form (rs_lowrate.cpp): the scalars alpha_K, beta_K of the
// W / C blocks, and the form on one symbol per position (host check); codes with at most
// kLowBlockMaxBlocks blocks
constexpr uint64_t kLowBlockMaxBlocks = 512;
void low_block_coefs(uint64_t k, uint64_t m, std::vector<uint16_t> &alpha, std::vector<uint16_t> &beta);
bool scalar_reconstruct_low_blocks(uint16_t *data, const uint16_t *par, const uint8_t *present, uint64_t k,
                                   uint64_t m);
void encode_low_map(uint64_t k, uint64_t m, uint32_t flags, jit::NetSpec &ns);

// -------------------------------------------------------- patterns (rs_patterns.cpp)
// Wide codes: the FFT kernel with per-stripe masks for the syndromes + the generic solve
// (pattern-agnostic: compiled once per code; also the batch syndrome path's cold form)
struct WpsSlot {
  std::shared_ptr<FftSlot> fft = std::make_shared<FftSlot>();
  std::shared_ptr<FftSlot> dec = std::make_shared<FftSlot>();  // fused FFT reconstruct (corrected multiply)
  std::shared_ptr<FftSlot> decb = std::make_shared<FftSlot>();  // the same, blocked unit walk (per-stripe blocks)
  std::mutex mu;
  bool solve_failed = false;
};
void wps_slot(int dev, uint64_t k, uint64_t m, uint32_t flags, std::shared_ptr<WpsSlot> &out);
const jit::Kernel *wps_solve_kernel(WpsSlot &ws);
// RS_AMD_FDEC: "0" never the fused FFT reconstruct, "1" whenever it applies, "auto"
// (default) unless the pattern's e x e network is loaded
int fdec_mode();
bool fdec_supports(uint64_t k, uint64_t m, uint64_t sb, uint32_t flags);
// RS_AMD_PDEC (default on): a reused wide-code pattern gets its pattern-compiled fused kernel
constexpr uint64_t kPdecMaxK = 256;  // pattern-compiled fused reconstruct: codes up to k = 256
bool pdec_enabled();
// Bounds on the per-pattern compiles (each 1-16 s of hipRTC on the one background worker, and
// a module that is never unloaded): a pattern is compiled in on its RS_AMD_PDEC_AFTER-th use
// (default 2, round 6: tools/pattern_stream.py; rs_reconstruct_warm at once), at most RS_AMD_PDEC_MAX patterns per code and
// device (default 32; later patterns keep the pattern-as-data kernel), and not while more
// than RS_AMD_PDEC_QUEUE jobs (default 2) wait on the worker (a later use retries).
uint32_t pdec_after();
size_t pdec_queue();
// admit the pattern `key` of code (dev, k, m) to the budget (true if already admitted)
bool pdec_admit(int dev, uint64_t k, uint64_t m, const std::string &key);
// exp, log, log_walsh in HBM (384 KiB per device)
int device_tables(int dev, const uint16_t **exp, const uint16_t **log, const uint16_t **lw);

}  // namespace host
}  // namespace rs
