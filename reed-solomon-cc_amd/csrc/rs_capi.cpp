// rs_capi.cpp — host codec and C ABI (include/reedsol.h) of librs_amd.so.
//
// Host-side mirror of root.zig: argument validation and error precedence of
// encode/decode/Encoder/Decoder/useHighRate, plan building (butterfly schedule
// + v_perm tables + erasure-locator evaluation) and kernel launches. Every
// device computation runs in rs_kernels.hip; there is no CPU compute path —
// without a gfx950 device the entry points return RS_ERR_NO_DEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/reedsol.h"
#include "rs_gf.hpp"
#include "rs_internal.hpp"
#include "rs_fftnet.hpp"
#include "rs_jit.hpp"
#include "rs_psyn.hpp"

using namespace rs;

namespace {

thread_local std::string t_last_error;

int fail(int status, const std::string &msg) {
  t_last_error = msg;
  return status;
}

int hip_fail(hipError_t e, const char *what) {
  return fail(RS_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr)                               \
  do {                                              \
    hipError_t e_ = (expr);                         \
    if (e_ != hipSuccess) return hip_fail(e_, #expr); \
  } while (0)

// ---------------------------------------------------------------- devices
std::mutex g_dev_mu;
std::map<int, int> g_dev_ok;  // device -> RS_OK / RS_ERR_NO_DEVICE

int current_device(int *dev) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(RS_ERR_NO_DEVICE, "no HIP device visible");
  HIP_TRY(hipGetDevice(dev));
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

// Low rate runs as maps of k x m GF(2^16) constants (passes of <= 64 outputs): the
// map size bounds the tables (96 B per entry) and the reconstruct's 16e x 16e solve.
constexpr uint64_t kLowRateMaxMap = 1ull << 16;
inline bool low_rate_ok(uint64_t k, uint64_t m) { return k * m <= kLowRateMaxMap; }

// Encoder.init / Decoder.init checks (root.zig:100-103, 198-201) + the tail panic (root.zig:385)
int check_codec(uint64_t k, uint64_t m, size_t shard_bytes) {
  const int hr = use_high_rate(k, m);
  if (hr < 0) return fail(-hr, "unsupported shard count (root.zig:397-415)");
  // low rate: the reference panics (root.zig:120); here maps with k * m <= 65536 (§8 f4)
  if (hr == 0 && !low_rate_ok(k, m))
    return fail(RS_ERR_LOW_RATE_UNSUPPORTED, "low-rate codec with original_count * recovery_count > 65536");
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

// ------------------------------------------------------------------ plans
struct DevBuf {
  void *p = nullptr;
  int dev = 0;
  ~DevBuf() {
    if (p) {
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

uint32_t async_after() {
  const char *e = std::getenv("RS_AMD_NET_ASYNC_AFTER");
  return e && *e ? static_cast<uint32_t>(std::max(1, std::atoi(e))) : 2u;
}

// Encodes of 1 / 2 KiB shards stay on the table kernels, which measured as fast or
// faster there (RS(10,4) 2 KiB 0.644 vs 0.678 ms, RS(4,2) 1 KiB 0.528 vs 0.541 ms,
// profiles/r01/sweep_small_shard_networks.jsonl); reconstructs take the networks
// (RS(10,4) 1 KiB losing 4: 1.16 -> 0.67 ms). RS_AMD_NET_SMALL_ENCODE=1 overrides.
// Encode maps past the synchronous network cap that no FFT kernel covers run as
// background-compiled networks (table kernels until they land): with the shared-input
// form for several tiles and one tile otherwise, every shape measured is faster than the
// table register kernel — RS(40,12) 1 MiB 4.08 -> 2.95 ms, RS(100,6) 2.85 -> 2.35 ms,
// RS(100,4) 2.49 -> 2.30 ms, RS(200,8) 2.75 -> 2.58 ms (profiles/r02/sweep_encode_async_net.jsonl).
bool encode_net_async(uint64_t k, uint64_t m) {
  const char *e = std::getenv("RS_AMD_NET_ASYNC_ENCODE");
  if (e && *e && std::strcmp(e, "0") == 0) return false;
  const char *sh = std::getenv("RS_AMD_NET_SHARED");
  if (sh && *sh && std::strcmp(sh, "0") == 0) return false;
  const char *lo = std::getenv("RS_AMD_NET_ASYNC_ENCODE_MIN_M");
  const uint64_t m_min = lo && *lo ? static_cast<uint64_t>(std::atoi(lo)) : 1;
  return m >= m_min && m <= jit::kMaxOut && !fftnet::supports(k, m, fftnet::kUnitBytes) &&
         jit::supports_async(static_cast<uint32_t>(k), static_cast<uint32_t>(m), jit::kUnitBytes);
}

bool encode_net_ok(uint64_t sb) {
  if (jit::net_pieces(sb) == 1) return true;
  const char *e = std::getenv("RS_AMD_NET_SMALL_ENCODE");
  return e && *e && std::strcmp(e, "0") != 0;
}

// A fallback to the table kernels is reported on stderr once per distinct reason.
void warn_once_per_reason(const char *what, const std::string &err) {
  static std::mutex mu;
  static std::set<std::string> seen;
  std::lock_guard<std::mutex> lk(mu);
  if (seen.insert(err.substr(0, 200)).second) std::fprintf(stderr, "%s%s\n", what, err.c_str());
}

// Bit-sliced FFT kernel of a plan (rs_fftnet.hpp): wide codes, compiled on first use.
struct FftSlot {
  std::mutex mu;
  bool failed[2] = {false, false};  // per variant: 2 KiB units of one stripe / of two 1 KiB stripes
  bool async = false;  // per-pattern kernels: background compile, the table encode meanwhile
  fftnet::Spec spec;
  fftnet::Spec spec_p2;  // the 1 KiB-shard variant (Spec::pieces 2), filled on first use
};

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
  const char *a = std::getenv("RS_AMD_FFT_ASYNC");
  const bool async = a && *a ? std::strcmp(a, "0") != 0 : slot.async;
  const jit::Kernel *k = fftnet::get(spec, async, err, pending);
  if (!k && !pending) {
    slot.failed[vi] = true;
    warn_once_per_reason("[rs_amd] bit-sliced FFT kernel unavailable, using table kernels: ", err);
  }
  return k;
}

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
  std::shared_ptr<FftSlot> syn_fft;  // the syndromes' encode on the bit-sliced FFT kernel (wide codes)
  std::shared_ptr<FftSlot> inv_fft;  // every original lost, k == m == chunk: the encode inverted
};

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

// Plan caches: least-recently-used entries past RS_AMD_PLAN_CACHE (default 4096 per
// kind) are dropped (a plan in use stays alive through its shared_ptr). g_plan_mu
// guards the maps only: plans are built without it (double-checked insertion; two
// threads racing on a new key may both build, the first insert wins).
size_t plan_cache_cap() {
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
  size_t size() const { return m.size(); }
};

std::mutex g_plan_mu;
PlanCache<EncodePlan> g_enc_plans;
PlanCache<DecodePlan> g_dec_plans;

int upload(const void *host, size_t bytes, int dev, std::shared_ptr<DevBuf> &out) {
  auto b = std::make_shared<DevBuf>();
  b->dev = dev;
  HIP_TRY(hipMalloc(&b->p, std::max<size_t>(bytes, 16)));
  HIP_TRY(hipMemcpy(b->p, host, bytes, hipMemcpyHostToDevice));
  out = b;
  return RS_OK;
}

// The encode as a k -> m map of GF(2)-linear 16x16 maps: images of every basis
// symbol of every data shard through Encoder.encode (root.zig:136-173).
void encode_map(uint64_t k, uint64_t m, uint32_t flags, jit::NetSpec &ns) {
  const bool d1 = flags & RS_FLAG_QUIRK_D1, d2 = flags & RS_FLAG_QUIRK_D2;
  ns.role = "encode";
  ns.n_in = static_cast<uint32_t>(k);
  ns.n_out = static_cast<uint32_t>(m);
  ns.src.clear();
  ns.images.assign(k * m * 16, 0);
  std::vector<uint16_t> in(k, 0), out(m);
  for (uint64_t t = 0; t < k; t++) {
    ns.src.push_back(static_cast<int32_t>(t));
    for (int b = 0; b < 16; b++) {
      in[t] = static_cast<uint16_t>(1u << b);
      scalar_encode(in.data(), k, m, d1, d2, out.data());
      for (uint64_t j = 0; j < m; j++) ns.images[(t * m + j) * 16 + b] = out[j];
    }
    in[t] = 0;
  }
}

// The reconstruct of one erasure pattern (root.zig:268-335) as an n_in -> e map.
// Inputs: every present original + the first e present recovery shards (exactly k:
// the unique restored data does not depend on which k). Under D1 the literal
// reconstruct is not a decoder, so its output depends on the pattern: keep ALL
// present shards then, exactly as the reference would receive them.
void reconstruct_map(uint64_t k, uint64_t m, uint32_t flags, const uint8_t *present, jit::NetSpec &ns) {
  const bool d1 = flags & RS_FLAG_QUIRK_D1;
  const uint64_t C = ceil_pow2(m), W = ceil_pow2(C + k);
  uint64_t present_count = 0;
  for (uint64_t i = 0; i < k + m; i++) present_count += present[i] ? 1 : 0;
  const uint64_t want = d1 ? present_count : k;
  std::vector<uint8_t> received(W, 0);
  std::vector<uint64_t> in_pos, out_pos;
  ns.role = "reconstruct";
  ns.src.clear();
  for (uint64_t i = 0; i < k; i++)
    if (present[i]) {
      received[C + i] = 1;
      in_pos.push_back(C + i);
      ns.src.push_back(static_cast<int32_t>(i));
    } else {
      out_pos.push_back(C + i);
    }
  for (uint64_t r = 0; r < m && in_pos.size() < want; r++)
    if (present[k + r]) {
      received[r] = 1;
      in_pos.push_back(r);
      ns.src.push_back(kSrcRecovery | static_cast<int32_t>(r));
    }
  std::vector<uint16_t> er(kOrder);
  erasure_logs(received.data(), k, m, er.data());
  const size_t n_in = in_pos.size(), n_out = out_pos.size();
  ns.n_in = static_cast<uint32_t>(n_in);
  ns.n_out = static_cast<uint32_t>(n_out);
  ns.images.assign(n_in * n_out * 16, 0);
  std::vector<uint16_t> sym(W);
  for (size_t t = 0; t < n_in; t++)
    for (int b = 0; b < 16; b++) {  // images of basis symbol 1<<b at input t
      std::fill(sym.begin(), sym.end(), 0);
      sym[in_pos[t]] = static_cast<uint16_t>(1u << b);
      scalar_reconstruct(sym.data(), received.data(), er.data(), k, m, d1);
      for (size_t j = 0; j < n_out; j++) ns.images[(t * n_out + j) * 16 + b] = sym[out_pos[j]];
    }
}

// root.zig:136-173 chunk schedule -> table block
int get_encode_plan(int dev, uint64_t k, uint64_t m, uint32_t flags, std::shared_ptr<EncodePlan> &out) {
  char key[128];
  std::snprintf(key, sizeof key, "%d/%llu/%llu/%u/%llu/%llu/%d", dev, (unsigned long long)k, (unsigned long long)m,
                flags, static_cast<unsigned long long>(jit::max_blocks()),
                static_cast<unsigned long long>(jit::max_async_blocks()), encode_net_async(k, m) ? 1 : 0);
  {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    if ((out = g_enc_plans.find(key))) return RS_OK;
  }
  const bool d1 = flags & RS_FLAG_QUIRK_D1, d2 = flags & RS_FLAG_QUIRK_D2;
  const uint64_t C = ceil_pow2(m);
  const std::vector<uint64_t> truncs = encode_chunk_truncs(k, m, d2);
  std::vector<RsTab> tabs;
  for (size_t j = 0; j < truncs.size(); j++) push_ifft_tabs(tabs, C, (j + 1) * C, d1);
  push_fft_tabs(tabs, C, 0, d1);
  auto plan = std::make_shared<EncodePlan>();
  int st = upload(tabs.data(), tabs.size() * sizeof(RsTab), dev, plan->buf);
  if (st) return st;
  plan->chunk = static_cast<uint32_t>(C);
  plan->n_chunks = static_cast<uint32_t>(truncs.size());
  plan->trunc_first = static_cast<uint32_t>(truncs.front());
  plan->trunc_last = static_cast<uint32_t>(truncs.back());
  plan->tabs_per_chunk = static_cast<uint32_t>(ifft_tab_count(C));
  plan->work = static_cast<uint32_t>((k + C - 1) / C * C);
  if (jit::supports(static_cast<uint32_t>(k), static_cast<uint32_t>(m), jit::kUnitBytes)) {
    encode_map(k, m, flags, plan->net->spec);
  } else if (encode_net_async(k, m)) {
    encode_map(k, m, flags, plan->net->spec);
    plan->net->async = true;
  }
  if (fftnet::supports(k, m, fftnet::kUnitBytes)) {
    plan->fft = std::make_shared<FftSlot>();
    plan->fft->spec.k = static_cast<uint32_t>(k);
    plan->fft->spec.m = static_cast<uint32_t>(m);
    plan->fft->spec.flags = flags;
  }
  std::lock_guard<std::mutex> lk(g_plan_mu);
  out = g_enc_plans.insert(key, plan);
  return RS_OK;
}

// Multiplies the FFT reconstruct performs for a pattern (plan-time estimate used to
// choose between the FFT kernels and the matrix kernel).
uint64_t fft_decode_mul_count(uint64_t k, uint64_t m, uint64_t present_count, uint64_t e) {
  const uint64_t C = ceil_pow2(m), end = C + k, W = ceil_pow2(C + k);
  const uint16_t *sk = tables().skew;
  auto live = [&](uint64_t idx) -> uint64_t { return idx < kModulus && sk[idx] != kModulus ? 1 : 0; };
  auto group = [&](uint64_t r, uint64_t d) {  // m01 + m23 over d pairs, m02 over 2d
    const uint64_t b = r + d - 1;
    return d * (live(b) + live(b + 2 * d)) + 2 * d * live(b + d);
  };
  uint64_t n = present_count + e;  // erasure masks + reveal (root.zig:292-303, 321-326)
  uint64_t d = 1;                  // IFFT, Generic.zig:80-147
  for (uint64_t d4 = 4; d4 <= W; d = d4, d4 <<= 2)
    for (uint64_t r = 0; r < end; r += d4) n += group(r, d);
  if (d < W) n += d * live(d - 1);
  uint64_t d4 = W;  // FFT, Generic.zig:15-78
  for (uint64_t dd = W >> 2; dd != 0; d4 = dd, dd >>= 2)
    for (uint64_t r = 0; r < end; r += d4) n += group(r, dd);
  if (d4 == 2)
    for (uint64_t r = 0; r < end; r += 2) n += live(r);
  return n;
}

const char *decode_mode_env() {
  const char *e = std::getenv("RS_AMD_DECODE");
  return e ? e : "auto";
}

constexpr uint32_t flags_none() { return 0; }

// Reconstruct kernel family for a pattern: 0 = FFT kernels (root.zig:268-335 as
// written), 1 = matrix (e <= 8, one wave), 2 = output-tiled matrix (e <= 64).
// The matrix kernels do k*e MACs at ~3/4 the cost of an FFT multiply (selectors
// shared across outputs); the FFT register kernels exist for W <= 32 only, beyond
// that the FFT path is the scratch-walking generic kernel (~10x slower per op).
int decode_kind(uint64_t k, uint64_t m, uint32_t flags, uint64_t e, uint64_t present_count, uint64_t sb) {
  (void)flags;
  const std::string mode = decode_mode_env();
  if (mode == "fft" || e == 0 || (k + m) > 4096) return 0;
  const uint64_t W = ceil_pow2(ceil_pow2(m) + k);
  const bool small_ok = e <= kMatrixMaxOut;
  const bool tiled_ok = e <= kMtileMaxOut && sb % 512 == 0;
  if (mode == "matrix") return small_ok ? 1 : tiled_ok ? 2 : 0;
  uint64_t fft_cost = 4 * fft_decode_mul_count(k, m, present_count, e);
  if (W > 32) fft_cost *= 10;  // generic kernel
  if (3 * k * e > fft_cost) return 0;
  return small_ok ? 1 : tiled_ok ? 2 : 0;
}

// Multiplies of one encode (root.zig:136-173) per 64-B column (live twiddles only).
uint64_t fft_encode_mul_count(uint64_t k, uint64_t m) {
  const uint64_t C = ceil_pow2(m);
  const uint16_t *sk = tables().skew;
  auto live = [&](uint64_t idx) -> uint64_t { return idx < kModulus && sk[idx] != kModulus ? 1 : 0; };
  auto group = [&](uint64_t b, uint64_t d) { return d * (live(b) + live(b + 2 * d)) + 2 * d * live(b + d); };
  const std::vector<uint64_t> truncs = encode_chunk_truncs(k, m, false);
  uint64_t n = 0;
  for (size_t j = 0; j < truncs.size(); j++) {  // IFFT per chunk, Generic.zig:80-147
    const uint64_t sd = (j + 1) * C;
    uint64_t d = 1;
    for (uint64_t d4 = 4; d4 <= C; d = d4, d4 <<= 2)
      for (uint64_t r = 0; r < truncs[j]; r += d4) n += group(r + d + sd - 1, d);
    if (d < C) n += d * live(d + sd - 1);
  }
  uint64_t d4 = C;  // FFT, Generic.zig:15-78
  for (uint64_t dd = C >> 2; dd != 0; d4 = dd, dd >>= 2)
    for (uint64_t r = 0; r < m; r += d4) n += group(r + dd - 1, dd);
  if (d4 == 2)
    for (uint64_t r = 0; r < m; r += 2) n += live(r);
  return n;
}

// a direct n_in -> e reconstruct map past the synchronous cap, within the background one
// A direct map past the synchronous cap, compiled in the background. For codes with an
// FFT kernel a large map loses to the syndrome path (FFT encode + e x e map): RS(200,55)
// losing 20 5.21 vs 3.90 ms, losing 14 3.56 vs 3.54, losing 8 2.61 vs 3.26 ms
// (profiles/r02/sweep_direct_vs_syndrome.jsonl), hence the n_in * e bound.
bool syndrome_pick(uint64_t k, uint64_t m, uint64_t e, uint32_t flags, uint64_t sb, const std::string &mode);
bool direct_net_async(uint64_t e, uint64_t n_in, uint64_t sb, const std::string &mode, uint64_t k, uint64_t m,
                      uint32_t flags) {
  if (mode == "auto" && fft_enabled() && fftnet::supports(k, m, sb) && n_in * e >= 2800 &&
      syndrome_pick(k, m, e, flags, sb, mode))
    return false;
  return (mode == "auto" || mode == "net") && jit::enabled() &&
         !jit::supports(static_cast<uint32_t>(n_in), static_cast<uint32_t>(e), sb) &&
         jit::supports_async(static_cast<uint32_t>(n_in), static_cast<uint32_t>(e), sb);
}

// Reconstruct by syndromes instead of the k x e matrix: worth it for wide codes
// with many erasures (RS(200,55) losing 55: 785 + 0.75*55^2 multiplies per column
// against 0.75*200*55). Needs the corrected multiply (under D1 the literal
// reconstruct is no inverse of the encode) and a fused (non-generic) encode kernel.
bool syndrome_pick(uint64_t k, uint64_t m, uint64_t e, uint32_t flags, uint64_t sb, const std::string &mode) {
  if ((flags & RS_FLAG_QUIRK_D1) || e == 0 || e > kMtileMaxOut || sb % 512) return false;
  if (choose_encode(k, m, sb, 4).variant == Variant::kGeneric) return false;
  if (mode == "syndrome") return true;
  if (mode != "auto") return false;
  const double direct = 0.75 * static_cast<double>(k) * e;
  const double syn = static_cast<double>(fft_encode_mul_count(k, m)) + 0.75 * static_cast<double>(e) * e;
  return syn < 0.7 * direct;
}

// x = A^-1 (p_R ^ Enc_R(d')): R = the first e received recovery rows, d' = the
// received data with the erased shards zeroed, A = the encode map from the erased
// columns to the rows R (e x e blocks of 16x16 GF(2) maps, invertible: the code is
// MDS). A is inverted as a 16e x 16e GF(2) matrix; the result is a matrix-kernel
// map whose input i is the syndrome rec[R_i] ^ Enc(d')[R_i] (kSrcXorScratch).
int syndrome_map(uint64_t k, uint64_t m, const uint8_t *present, jit::NetSpec &ns) {
  std::vector<uint64_t> E, Rr;
  for (uint64_t i = 0; i < k; i++)
    if (!present[i]) E.push_back(i);
  for (uint64_t r = 0; r < m && Rr.size() < E.size(); r++)
    if (present[k + r]) Rr.push_back(r);
  const size_t e = E.size();
  if (Rr.size() < e) return fail(RS_ERR_NOT_ENOUGH_SHARDS, "fewer than original_count shards present");
  const size_t N = 16 * e, words = (2 * N + 63) / 64;
  // augmented [A | I], row (16 j + c) = bit c of the row-R_j output, column (16 t + b) = basis b of column E_t
  std::vector<std::vector<uint64_t>> M(N, std::vector<uint64_t>(words, 0));
  std::vector<uint16_t> in(k, 0), out(m);
  for (size_t t = 0; t < e; t++)
    for (int b = 0; b < 16; b++) {
      in[E[t]] = static_cast<uint16_t>(1u << b);
      scalar_encode(in.data(), k, m, false, false, out.data());
      in[E[t]] = 0;
      const size_t col = 16 * t + b;
      for (size_t j = 0; j < e; j++)
        for (int c = 0; c < 16; c++)
          if (out[Rr[j]] >> c & 1) M[16 * j + c][col / 64] |= 1ull << (col % 64);
    }
  for (size_t r = 0; r < N; r++) M[r][(N + r) / 64] |= 1ull << ((N + r) % 64);
  for (size_t col = 0; col < N; col++) {  // Gauss-Jordan over GF(2)
    size_t piv = col;
    while (piv < N && !(M[piv][col / 64] >> (col % 64) & 1)) piv++;
    if (piv == N) return fail(RS_ERR_DEVICE, "syndrome matrix singular");
    std::swap(M[piv], M[col]);
    for (size_t r = 0; r < N; r++)
      if (r != col && (M[r][col / 64] >> (col % 64) & 1))
        for (size_t w = 0; w < words; w++) M[r][w] ^= M[col][w];
  }
  // B = A^-1: x bit (16 j + c) = XOR over s bits (16 i + b) of B[16 j + c][16 i + b]
  ns.role = "syndrome";
  ns.n_in = static_cast<uint32_t>(e);
  ns.n_out = static_cast<uint32_t>(e);
  ns.src.assign(e, 0);
  ns.images.assign(e * e * 16, 0);
  for (size_t i = 0; i < e; i++) {
    ns.src[i] = kSrcXorScratch | kSrcRecovery | static_cast<int32_t>(Rr[i]);
    for (int b = 0; b < 16; b++) {
      const size_t col = N + 16 * i + b;
      for (size_t j = 0; j < e; j++)
        for (int c = 0; c < 16; c++)
          if (M[16 * j + c][col / 64] >> (col % 64) & 1) ns.images[(i * e + j) * 16 + b] |= static_cast<uint16_t>(1u << c);
    }
  }
  return RS_OK;
}

// root.zig:268-335 erasure pattern -> evalPoly -> masks and table block (FFT
// kernels), or -> the reconstruct's linear map as an e x k matrix (matrix kernel).
int get_decode_plan(int dev, uint64_t k, uint64_t m, uint64_t sb, uint32_t flags, const uint8_t *present,
                    std::shared_ptr<DecodePlan> &out) {
  const std::string mode = decode_mode_env();
  std::string key = std::to_string(dev) + "/" + std::to_string(k) + "/" + std::to_string(m) + "/" +
                    std::to_string(flags) + "/" + mode + "/" + std::to_string(sb % 512 == 0) + "/" +
                    std::to_string(jit::enabled() && jit::shard_ok(sb)) + "/" +
                    std::to_string(fft_enabled() && fftnet::supports(k, m, sb)) + "/" +
                    std::to_string(jit::max_blocks()) + "/" + std::to_string(jit::max_async_blocks()) + "/";
  key.reserve(key.size() + k + m);
  for (uint64_t i = 0; i < k + m; i++) key.push_back(present[i] ? '1' : '0');
  {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    if ((out = g_dec_plans.find(key))) return RS_OK;
  }
  const bool d1 = flags & RS_FLAG_QUIRK_D1;
  const uint64_t C = ceil_pow2(m), end = C + k, W = ceil_pow2(C + k);
  uint64_t e = 0, present_count = 0;
  for (uint64_t i = 0; i < k; i++) e += present[i] ? 0 : 1;
  for (uint64_t i = 0; i < k + m; i++) present_count += present[i] ? 1 : 0;
  int kind = decode_kind(k, m, flags, e, present_count, sb);
  // bit-sliced network (rs_jit.hpp): the same e x k map as the matrix kernels at a
  // fraction of their VALU cost, so preferred whenever it applies (modes auto / net)
  const uint64_t n_in_want = d1 ? present_count : k;
  const bool use_net = (mode == "auto" || mode == "net") && jit::enabled() &&
                       jit::supports(static_cast<uint32_t>(n_in_want), static_cast<uint32_t>(e), sb);
  if (use_net && kind == 0) kind = e <= kMatrixMaxOut ? 1 : 2;  // table kernels stay as the fallback
  // past the synchronous cap: the same map compiled in the background, the matrix
  // kernel meanwhile (RS(200,55) losing 8: 400 blocks, against syndrome + encode)
  const bool use_net_async = !use_net && kind != 0 && direct_net_async(e, n_in_want, sb, mode, k, m, flags);
  const bool use_syn = !use_net && !use_net_async && syndrome_pick(k, m, e, flags, sb, mode);
  if (use_syn) kind = e <= kMatrixMaxOut ? 1 : 2;
  // the syndromes' e x e map as a network too (its table kernel stays the fallback)
  const bool syn_net = use_syn && (mode == "auto" || mode == "net" || mode == "syndrome") && jit::enabled() &&
                       jit::supports_async(static_cast<uint32_t>(e), static_cast<uint32_t>(e), sb);
  const bool use_matrix = kind != 0;

  auto plan = std::make_shared<DecodePlan>();
  plan->work = static_cast<uint32_t>(W);
  plan->chunk = static_cast<uint32_t>(C);
  plan->trunc = static_cast<uint32_t>(end);
  // every original lost and every recovery shard present, k == m == chunk: the data are
  // FFT_C(IFFT_0(recovery)) (rs_fftnet.hpp Spec::inverse); the plan's other kernels stay
  // the fallback
  // (corrected multiply only: under D1 the literal reconstruct is no inverse of the encode,
  // so its output is not the data and must follow root.zig:268-335 as written)
  if (e == k && present_count == m && !d1 && (mode == "auto" || mode == "net") && fft_enabled() &&
      fftnet::supports_inverse(k, m, sb)) {
    plan->inv_fft = std::make_shared<FftSlot>();
    plan->inv_fft->spec.k = static_cast<uint32_t>(k);
    plan->inv_fft->spec.m = static_cast<uint32_t>(m);
    plan->inv_fft->spec.flags = flags;
    plan->inv_fft->spec.inverse = true;
  }

  if (use_matrix) {
    jit::NetSpec map;
    if (use_syn) {
      int st = syndrome_map(k, m, present, map);
      if (st) return st;
      std::vector<uint32_t> bits((k + 31) / 32, 0);
      for (uint64_t i = 0; i < k; i++)
        if (!present[i]) bits[i / 32] |= 1u << (i % 32);
      if ((st = upload(bits.data(), bits.size() * sizeof(uint32_t), dev, plan->skip))) return st;
      plan->syndrome = true;
      if (fft_enabled() && fftnet::supports(k, m, sb)) {
        // Enc(d') on the FFT kernel: erased data shards read as zero, only the rows R stored
        plan->syn_fft = std::make_shared<FftSlot>();
        plan->syn_fft->async = true;
        fftnet::Spec &fs = plan->syn_fft->spec;
        fs.k = static_cast<uint32_t>(k);
        fs.m = static_cast<uint32_t>(m);
        fs.flags = RS_FLAG_CORRECTED;
        fs.skip.assign(k, 0);
        for (uint64_t i = 0; i < k; i++) fs.skip[i] = present[i] ? 0 : 1;
        fs.out_mode.assign(m, fftnet::kOutNone);
        for (int32_t src : map.src) fs.out_mode[src & kSrcIndexMask] = fftnet::kOutStore;
      }
    } else {
      reconstruct_map(k, m, flags, present, map);
    }
    const std::vector<int32_t> &src = map.src;
    const std::vector<uint16_t> &img = map.images;
    const size_t n_in = map.n_in, n_out = map.n_out;
    // rows of n_out tables (kind 1) or padded to kMtileMaxOut zero tables (kind 2)
    const size_t row = kind == 2 ? kMtileMaxOut : n_out;
    std::vector<RsTab> tabs(n_in * row);
    for (size_t t = 0; t < n_in; t++)
      for (size_t j = 0; j < n_out; j++) tabs[t * row + j] = make_tab_from_images(&img[(t * n_out + j) * 16]);
    std::vector<uint8_t> blob(tabs.size() * sizeof(RsTab) + n_in * sizeof(int32_t));
    std::memcpy(blob.data(), tabs.data(), tabs.size() * sizeof(RsTab));
    std::memcpy(blob.data() + tabs.size() * sizeof(RsTab), src.data(), n_in * sizeof(int32_t));
    int st = upload(blob.data(), blob.size(), dev, plan->buf);
    if (st) return st;
    plan->matrix = true;
    plan->tiled = kind == 2;
    if (use_net || use_net_async || syn_net) {
      plan->net = std::make_shared<NetSlot>();
      plan->net->async = !jit::supports(map.n_in, map.n_out, sb);
      plan->net->spec = std::move(map);
    }
    plan->e = static_cast<uint32_t>(n_out);
    plan->n_in = static_cast<uint32_t>(n_in);
    plan->off_mat = 0;
    plan->off_src = tabs.size() * sizeof(RsTab);
    std::lock_guard<std::mutex> lk(g_plan_mu);
    out = g_dec_plans.insert(key, plan);
    return RS_OK;
  }

  std::vector<uint8_t> received(W, 0);
  for (uint64_t i = 0; i < m; i++) received[i] = present[k + i] ? 1 : 0;
  for (uint64_t i = 0; i < k; i++) received[C + i] = present[i] ? 1 : 0;
  std::vector<uint16_t> er(kOrder, 0);
  erasure_logs(received.data(), k, m, er.data());  // root.zig:277-289

  std::vector<RsTab> tabs;
  push_ifft_tabs(tabs, W, 0, d1);
  const size_t n_ifft = tabs.size();
  push_fft_tabs(tabs, W, 0, d1);
  const size_t n_fft = tabs.size() - n_ifft;
  std::vector<int32_t> src(W, -1), dst(W, -1);
  std::vector<RsTab> pre(W), post(W);
  uint32_t ne = 0;
  for (uint64_t p = 0; p < W; p++) {
    if (p < m && received[p]) {
      src[p] = kSrcRecovery | static_cast<int32_t>(p);
      pre[p] = make_tab(er[p], d1);
    } else if (p >= C && p < end && received[p]) {
      src[p] = static_cast<int32_t>(p - C);
      pre[p] = make_tab(er[p], d1);
    }
    if (p >= C && p < end && !received[p]) {
      dst[p] = static_cast<int32_t>(ne++);
      post[p] = make_tab(static_cast<uint16_t>(kModulus - er[p]), d1);  // root.zig:321-326
    }
  }
  tabs.insert(tabs.end(), pre.begin(), pre.end());
  tabs.insert(tabs.end(), post.begin(), post.end());
  std::vector<uint8_t> blob(tabs.size() * sizeof(RsTab) + 2 * W * sizeof(int32_t));
  std::memcpy(blob.data(), tabs.data(), tabs.size() * sizeof(RsTab));
  const size_t off_src = tabs.size() * sizeof(RsTab), off_dst = off_src + W * sizeof(int32_t);
  std::memcpy(blob.data() + off_src, src.data(), W * sizeof(int32_t));
  std::memcpy(blob.data() + off_dst, dst.data(), W * sizeof(int32_t));
  int st = upload(blob.data(), blob.size(), dev, plan->buf);
  if (st) return st;
  plan->e = ne;
  plan->off_fft = n_ifft * sizeof(RsTab);
  plan->off_pre = (n_ifft + n_fft) * sizeof(RsTab);
  plan->off_post = plan->off_pre + W * sizeof(RsTab);
  plan->off_src = off_src;
  plan->off_dst = off_dst;
  std::lock_guard<std::mutex> lk(g_plan_mu);
  out = g_dec_plans.insert(key, plan);
  return RS_OK;
}

constexpr uint64_t kScratchCap = 1ull << 30;  // generic path: scratch per launch

// ------------------------------------------------------- low-rate codec (§8 f4)
// The reference panics on low rate (root.zig:119-121, 226-228). Here the encode
// is reed-solomon-simd's low-rate encoder (rs_gf.hpp scalar_encode_low; parity
// unpinned: no reference output exists) and a reconstruct is the unique MDS
// solution, derived by linear algebra from the encode map. Both run as maps on
// the network kernels, or on the table matrix kernels in groups of <= 8 outputs.
bool is_low_rate(uint64_t k, uint64_t m) { return use_high_rate(k, m) == 0; }

void encode_low_map(uint64_t k, uint64_t m, uint32_t flags, jit::NetSpec &ns) {
  const bool d1 = flags & RS_FLAG_QUIRK_D1;
  ns.role = "encode_low";
  ns.n_in = static_cast<uint32_t>(k);
  ns.n_out = static_cast<uint32_t>(m);
  ns.src.clear();
  ns.images.assign(k * m * 16, 0);
  std::vector<uint16_t> in(k, 0), out(m);
  for (uint64_t t = 0; t < k; t++) {
    ns.src.push_back(static_cast<int32_t>(t));
    for (int b = 0; b < 16; b++) {
      in[t] = static_cast<uint16_t>(1u << b);
      scalar_encode_low(in.data(), k, m, d1, out.data());
      for (uint64_t j = 0; j < m; j++) ns.images[(t * m + j) * 16 + b] = out[j];
    }
    in[t] = 0;
  }
}

// Reconstruct of a systematic linear code with encode map G (G.images[(t*m + r)*16 + b]
// = parity r of basis b at data t): with E the erased data, P the present data and R
// the first e present recovery rows, p_R = G_RE x + G_RP d_P, so
// x = G_RE^-1 (p_R + G_RP d_P): a map from [d_P, p_R] to x (16e x 16e GF(2) solve).
int linear_decode_map(uint64_t k, uint64_t m, const jit::NetSpec &G, const uint8_t *present, const char *role,
                      jit::NetSpec &ns) {
  std::vector<uint64_t> E, P, Rr;
  for (uint64_t i = 0; i < k; i++) (present[i] ? P : E).push_back(i);
  for (uint64_t r = 0; r < m && Rr.size() < E.size(); r++)
    if (present[k + r]) Rr.push_back(r);
  const size_t e = E.size(), np = P.size();
  if (Rr.size() < e) return fail(RS_ERR_NOT_ENOUGH_SHARDS, "fewer than original_count shards present");
  const size_t N = 16 * e, cols = N + 16 * np + N, words = (cols + 63) / 64;
  auto g = [&](uint64_t t, uint64_t r, int b) { return G.images[(t * m + r) * 16 + b]; };
  std::vector<std::vector<uint64_t>> M(N, std::vector<uint64_t>(words, 0));
  auto set = [&](size_t row, size_t col) { M[row][col / 64] |= 1ull << (col % 64); };
  for (size_t j = 0; j < e; j++)
    for (int c = 0; c < 16; c++) {
      const size_t row = 16 * j + c;
      for (size_t t = 0; t < e; t++)  // [G_RE | G_RP | I]
        for (int b = 0; b < 16; b++)
          if (g(E[t], Rr[j], b) >> c & 1) set(row, 16 * t + b);
      for (size_t t = 0; t < np; t++)
        for (int b = 0; b < 16; b++)
          if (g(P[t], Rr[j], b) >> c & 1) set(row, N + 16 * t + b);
      set(row, N + 16 * np + row);
    }
  for (size_t col = 0; col < N; col++) {  // Gauss-Jordan over GF(2)
    size_t piv = col;
    while (piv < N && !(M[piv][col / 64] >> (col % 64) & 1)) piv++;
    if (piv == N) return fail(RS_ERR_DEVICE, "decode matrix singular");
    std::swap(M[piv], M[col]);
    for (size_t r = 0; r < N; r++)
      if (r != col && (M[r][col / 64] >> (col % 64) & 1))
        for (size_t w = 0; w < words; w++) M[r][w] ^= M[col][w];
  }
  // x = [G_RE^-1 G_RP | G_RE^-1] [d_P; p_R]
  ns.role = role;
  ns.n_in = static_cast<uint32_t>(np + e);
  ns.n_out = static_cast<uint32_t>(e);
  ns.src.clear();
  for (uint64_t i : P) ns.src.push_back(static_cast<int32_t>(i));
  for (uint64_t r : Rr) ns.src.push_back(kSrcRecovery | static_cast<int32_t>(r));
  ns.images.assign(static_cast<size_t>(ns.n_in) * e * 16, 0);
  for (size_t i = 0; i < ns.n_in; i++)
    for (int b = 0; b < 16; b++) {
      const size_t col = N + 16 * i + b;
      for (size_t j = 0; j < e; j++)
        for (int c = 0; c < 16; c++)
          if (M[16 * j + c][col / 64] >> (col % 64) & 1) ns.images[(i * e + j) * 16 + b] |= static_cast<uint16_t>(1u << c);
    }
  return RS_OK;
}

// A map on the device, in passes of <= 64 outputs (jit::kMaxOut; every pass reads
// all inputs): per pass the network kernel when it fits, else the table matrix
// kernels over groups of <= 8 outputs (blocks [group][n_in][E_g] of tables + src).
struct MapPlan {
  std::shared_ptr<DevBuf> buf;
  uint32_t n_in = 0, n_out = 0;
  std::vector<size_t> group_off;  // byte offset of each group's table block
  size_t off_src = 0;
  std::vector<std::shared_ptr<NetSlot>> net;  // per pass: outputs [64 p, 64 p + 64)
};

inline uint32_t map_passes(uint32_t n_out) { return (n_out + jit::kMaxOut - 1) / jit::kMaxOut; }
// every pass of an n_in x n_out map has a network form (the first pass is the widest)
bool map_net_ok(uint64_t n_in, uint64_t n_out, uint64_t sb) {
  return jit::enabled() && n_out > 0 &&
         jit::supports_async(static_cast<uint32_t>(n_in), static_cast<uint32_t>(std::min<uint64_t>(n_out, jit::kMaxOut)), sb);
}
PlanCache<MapPlan> g_map_plans;

int build_map_plan(int dev, jit::NetSpec &&spec, std::shared_ptr<MapPlan> &out) {
  auto p = std::make_shared<MapPlan>();
  p->n_in = spec.n_in;
  p->n_out = spec.n_out;
  std::vector<RsTab> tabs;
  for (uint32_t j0 = 0; j0 < spec.n_out; j0 += kMatrixMaxOut) {
    const uint32_t eg = std::min<uint32_t>(kMatrixMaxOut, spec.n_out - j0);
    p->group_off.push_back(tabs.size() * sizeof(RsTab));
    for (uint32_t t = 0; t < spec.n_in; t++)
      for (uint32_t j = 0; j < eg; j++)
        tabs.push_back(make_tab_from_images(&spec.images[(static_cast<size_t>(t) * spec.n_out + j0 + j) * 16]));
  }
  std::vector<uint8_t> blob(tabs.size() * sizeof(RsTab) + spec.n_in * sizeof(int32_t));
  std::memcpy(blob.data(), tabs.data(), tabs.size() * sizeof(RsTab));
  std::memcpy(blob.data() + tabs.size() * sizeof(RsTab), spec.src.data(), spec.n_in * sizeof(int32_t));
  p->off_src = tabs.size() * sizeof(RsTab);
  int st = upload(blob.data(), blob.size(), dev, p->buf);
  if (st) return st;
  for (uint32_t j0 = 0; j0 < spec.n_out; j0 += jit::kMaxOut) {
    const uint32_t len = std::min<uint32_t>(jit::kMaxOut, spec.n_out - j0);
    auto slot = std::make_shared<NetSlot>();
    slot->async = !jit::supports(p->n_in, len, jit::kUnitBytes);  // larger maps: background compile
    jit::NetSpec &ps = slot->spec;
    ps.role = spec.role;
    ps.n_in = spec.n_in;
    ps.n_out = len;
    ps.src = spec.src;
    if (len == spec.n_out) {
      ps.images = std::move(spec.images);
    } else {
      ps.images.resize(static_cast<size_t>(spec.n_in) * len * 16);
      for (uint32_t t = 0; t < spec.n_in; t++)
        std::memcpy(&ps.images[static_cast<size_t>(t) * len * 16],
                    &spec.images[(static_cast<size_t>(t) * spec.n_out + j0) * 16], len * 16 * sizeof(uint16_t));
    }
    p->net.push_back(std::move(slot));
  }
  out = p;
  return RS_OK;
}

int run_map_pass(const MapPlan &p, uint32_t pi, bool net_ok, uint64_t sb, uint64_t n, const uint8_t *b0, uint64_t s0,
                 const uint8_t *b1, uint64_t s1, uint8_t *out, uint64_t so, int max_nv, hipStream_t s);

// out[j] = sum_i map_ij(in_i) for every stripe; inputs per src (buffer 0 / 1).
int run_map(const MapPlan &p, uint64_t sb, uint64_t n, const uint8_t *b0, uint64_t s0, const uint8_t *b1, uint64_t s1,
            uint8_t *out, uint64_t so, int max_nv, hipStream_t s) {
  if (!b0) b0 = b1;
  if (!b1) b1 = b0;
  const bool net_ok = max_nv == 4 && map_net_ok(p.n_in, p.n_out, sb);
  for (uint32_t pi = 0; pi < p.net.size(); pi++)
    if (int st = run_map_pass(p, pi, net_ok, sb, n, b0, s0, b1, s1, out, so, max_nv, s)) return st;
  return RS_OK;
}

int run_map_pass(const MapPlan &p, uint32_t pi, bool net_ok, uint64_t sb, uint64_t n, const uint8_t *b0, uint64_t s0,
                 const uint8_t *b1, uint64_t s1, uint8_t *out, uint64_t so, int max_nv, hipStream_t s) {
  const uint32_t p0 = pi * jit::kMaxOut, p1 = std::min<uint32_t>(p.n_out, p0 + jit::kMaxOut);
  if (net_ok)
    if (const jit::Kernel *nk = net_kernel(*p.net[pi], sb)) {
      HIP_TRY(jit::launch(*nk, b0, s0, b1, s1, out + static_cast<uint64_t>(p0) * sb, so, sb, n, s));
      return RS_OK;
    }
  const uint8_t *base = static_cast<const uint8_t *>(p.buf->p);
  for (size_t g = p0 / kMatrixMaxOut; g < p.group_off.size() && g * kMatrixMaxOut < p1; g++) {
    const uint32_t j0 = static_cast<uint32_t>(g * kMatrixMaxOut);
    const uint32_t eg = std::min<uint32_t>(kMatrixMaxOut, p.n_out - j0);
    const KernelChoice kc = choose_decode_matrix(eg, sb, max_nv);
    DecodeArgs a{};
    a.orig = b0;
    a.orig_stripe_stride = s0;
    a.rec = b1;
    a.rec_stripe_stride = s1;
    a.out = out + static_cast<uint64_t>(j0) * sb;
    a.out_stripe_stride = so;
    a.shard_bytes = sb;
    a.tab_mat = reinterpret_cast<const RsTab *>(base + p.group_off[g]);
    a.pos_src = reinterpret_cast<const int32_t *>(base + p.off_src);
    a.n_in = p.n_in;
    a.n_out = eg;
    a.contig = contig_ok(sb, kc.nv);
    a.n_stripes = n;
    // launch_decode advances these per 65535-stripe slice: keep them valid
    a.tab_pre = a.tab_post = a.tab_mat;
    a.pos_dst = a.pos_src;
    HIP_TRY(launch_decode(kc, a, s));
  }
  return RS_OK;
}

int get_low_encode_plan(int dev, uint64_t k, uint64_t m, uint32_t flags, std::shared_ptr<MapPlan> &out) {
  const std::string key = "lowenc/" + std::to_string(dev) + "/" + std::to_string(k) + "/" + std::to_string(m) + "/" +
                          std::to_string(flags & RS_FLAG_QUIRK_D1);
  {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    if ((out = g_map_plans.find(key))) return RS_OK;
  }
  jit::NetSpec spec;
  encode_low_map(k, m, flags, spec);
  int st = build_map_plan(dev, std::move(spec), out);
  if (st) return st;
  std::lock_guard<std::mutex> lk(g_plan_mu);
  out = g_map_plans.insert(key, out);
  return RS_OK;
}

int low_decode_map(uint64_t k, uint64_t m, uint32_t flags, const uint8_t *present, jit::NetSpec &ns) {
  jit::NetSpec G;
  encode_low_map(k, m, flags, G);
  return linear_decode_map(k, m, G, present, "reconstruct_low", ns);
}

int get_low_decode_plan(int dev, uint64_t k, uint64_t m, uint32_t flags, const uint8_t *present,
                        std::shared_ptr<MapPlan> &out) {
  std::string key = "lowdec/" + std::to_string(dev) + "/" + std::to_string(k) + "/" + std::to_string(m) + "/" +
                    std::to_string(flags & RS_FLAG_QUIRK_D1) + "/";
  for (uint64_t i = 0; i < k + m; i++) key.push_back(present[i] ? '1' : '0');
  {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    if ((out = g_map_plans.find(key))) return RS_OK;
  }
  jit::NetSpec spec;
  int st = low_decode_map(k, m, flags, present, spec);
  if (st) return st;
  if ((st = build_map_plan(dev, std::move(spec), out))) return st;
  std::lock_guard<std::mutex> lk(g_plan_mu);
  out = g_map_plans.insert(key, out);
  return RS_OK;
}

// ---------------------------------------------------------- shard tails
// Batches whose shard_bytes is not a multiple of 64 run on padded copies
// ([stripe][shard][ceil(sb/64)*64], tail chunk in the reference's layout) in
// slices of <= 1 GiB, then the outputs are unpadded.
constexpr uint64_t kTailSliceBytes = 1ull << 30;

int pad_shards(const uint8_t *src, uint64_t src_stripe_stride, uint64_t sb, uint8_t *dst, uint64_t dst_stripe_stride,
               uint64_t psb, uint64_t n, hipStream_t s) {
  const uint64_t whole = sb / 64 * 64;
  if (whole) HIP_TRY(hipMemcpy2DAsync(dst, dst_stripe_stride, src, src_stripe_stride, whole, n, hipMemcpyDeviceToDevice, s));
  (void)psb;
  HIP_TRY(launch_tail_pack(src, src_stripe_stride, dst, dst_stripe_stride, sb, n, false, s));
  return RS_OK;
}

int unpad_shards(const uint8_t *src, uint64_t src_stripe_stride, uint64_t sb, uint8_t *dst, uint64_t dst_stripe_stride,
                 uint64_t n, hipStream_t s) {
  const uint64_t whole = sb / 64 * 64;
  if (whole) HIP_TRY(hipMemcpy2DAsync(dst, dst_stripe_stride, src, src_stripe_stride, whole, n, hipMemcpyDeviceToDevice, s));
  HIP_TRY(launch_tail_pack(src, src_stripe_stride, dst, dst_stripe_stride, sb, n, true, s));
  return RS_OK;
}

}  // namespace

extern "C" int rs_encode_batch_dev(uint64_t, uint64_t, size_t, uint64_t, const void *, uint64_t, void *, uint64_t,
                                   uint32_t, rs_stream_t);
extern "C" int rs_reconstruct_batch_dev(uint64_t, uint64_t, size_t, uint64_t, const uint8_t *, const void *, uint64_t,
                                        const void *, uint64_t, void *, uint64_t, uint32_t, rs_stream_t);

namespace {

int encode_tail(uint64_t k, uint64_t m, uint64_t sb, uint64_t n, const uint8_t *orig, uint64_t ostride, uint8_t *rec,
                uint64_t rstride, uint32_t flags, hipStream_t s) {
  const uint64_t psb = (sb + 63) / 64 * 64;
  const uint64_t cap = std::max<uint64_t>(1, std::min<uint64_t>(n, kTailSliceBytes / ((k + m) * psb)));
  void *buf = nullptr;
  HIP_TRY(hipMallocAsync(&buf, cap * (k + m) * psb, s));
  uint8_t *pin = static_cast<uint8_t *>(buf), *pout = pin + cap * k * psb;
  int st = RS_OK;
  for (uint64_t s0 = 0; st == RS_OK && s0 < n; s0 += cap) {
    const uint64_t cnt = std::min(cap, n - s0);
    for (uint64_t i = 0; st == RS_OK && i < k; i++)
      st = pad_shards(orig + s0 * ostride + i * sb, ostride, sb, pin + i * psb, k * psb, psb, cnt, s);
    if (st == RS_OK) st = rs_encode_batch_dev(k, m, psb, cnt, pin, 0, pout, 0, flags, s);
    for (uint64_t r = 0; st == RS_OK && r < m; r++)
      st = unpad_shards(pout + r * psb, m * psb, sb, rec + s0 * rstride + r * sb, rstride, cnt, s);
  }
  (void)hipFreeAsync(buf, s);
  return st;
}

int reconstruct_tail(uint64_t k, uint64_t m, uint64_t sb, uint64_t n, const uint8_t *present, uint64_t e,
                     const uint8_t *orig, uint64_t ostride, const uint8_t *rec, uint64_t rstride, uint8_t *out,
                     uint64_t outstride, uint32_t flags, hipStream_t s) {
  const uint64_t psb = (sb + 63) / 64 * 64;
  const uint64_t cap = std::max<uint64_t>(1, std::min<uint64_t>(n, kTailSliceBytes / ((k + m + e) * psb)));
  void *buf = nullptr;
  HIP_TRY(hipMallocAsync(&buf, cap * (k + m + e) * psb, s));
  uint8_t *po = static_cast<uint8_t *>(buf), *pr = po + cap * k * psb, *pout = pr + cap * m * psb;
  int st = RS_OK;
  for (uint64_t s0 = 0; st == RS_OK && s0 < n; s0 += cap) {
    const uint64_t cnt = std::min(cap, n - s0);
    for (uint64_t i = 0; st == RS_OK && i < k; i++)  // only present shards are read
      if (present[i]) st = pad_shards(orig + s0 * ostride + i * sb, ostride, sb, po + i * psb, k * psb, psb, cnt, s);
    for (uint64_t i = 0; st == RS_OK && i < m; i++)
      if (present[k + i])
        st = pad_shards(rec + s0 * rstride + i * sb, rstride, sb, pr + i * psb, m * psb, psb, cnt, s);
    if (st == RS_OK) st = rs_reconstruct_batch_dev(k, m, psb, cnt, present, po, 0, pr, 0, pout, 0, flags, s);
    for (uint64_t j = 0; st == RS_OK && j < e; j++)
      st = unpad_shards(pout + j * psb, e * psb, sb, out + s0 * outstride + j * sb, outstride, cnt, s);
  }
  (void)hipFreeAsync(buf, s);
  return st;
}

}  // namespace

// ===================================================================== ABI
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

const char *rs_last_error(void) { return t_last_error.c_str(); }

int rs_use_high_rate(uint64_t k, uint64_t m) { return use_high_rate(k, m); }

const uint16_t *rs_table_exp(void) { return tables().exp; }
const uint16_t *rs_table_log(void) { return tables().log; }
const uint16_t *rs_table_skew(void) { return tables().skew; }
const uint16_t *rs_table_log_walsh(void) { return tables().log_walsh; }

// Names of the kernels a call with 16-byte aligned buffers would run (bit-sliced
// networks: "net_<role>_i<inputs>_o<outputs>"; the hipRTC symbol rs_net_... adds a content hash).
static const char *net_name(const char *role, uint64_t n_in, uint64_t n_out) {
  thread_local std::string name;
  name = std::string("net_") + role + "_i" + std::to_string(n_in) + "_o" + std::to_string(n_out);
  return name.c_str();
}

const char *rs_encode_kernel_name(uint64_t k, uint64_t m, size_t sb) {
  if (is_low_rate(k, m)) {
    if (map_net_ok(k, m, sb)) return net_name("encode_low", k, m);
    return "lowrate_matrix";
  }
  if (fft_enabled() && fftnet::supports(k, m, sb)) return net_name("fft_encode", k, m);
  if (jit::enabled() && encode_net_ok(sb) &&
      (jit::supports(static_cast<uint32_t>(k), static_cast<uint32_t>(m), sb) ||
       (encode_net_async(k, m) && jit::supports_async(static_cast<uint32_t>(k), static_cast<uint32_t>(m), sb) &&
        jit::net_pieces(sb) == 1)))
    return net_name("encode", k, m);
  return choose_encode(k, m, sb, 4).name;
}
const char *rs_reconstruct_kernel_name(uint64_t k, uint64_t m, size_t sb, const uint8_t *present) {
  std::vector<uint8_t> def;
  if (!present) {
    def.assign(k + m, 1);
    for (uint64_t i = 0; i < std::min(k, m); i++) def[i] = 0;
    present = def.data();
  }
  uint64_t e = 0, have = 0;
  for (uint64_t i = 0; i < k; i++) e += present[i] ? 0 : 1;
  for (uint64_t i = 0; i < k + m; i++) have += present[i] ? 1 : 0;
  if (is_low_rate(k, m)) {
    if (map_net_ok(k, e, sb)) return net_name("reconstruct_low", k, e);
    return "lowrate_matrix";
  }
  const std::string mode = decode_mode_env();
  if (e == k && have == m && (mode == "auto" || mode == "net") && fft_enabled() && fftnet::supports_inverse(k, m, sb))
    return net_name("fft_inverse", m, k);
  if ((mode == "auto" || mode == "net") && jit::enabled() &&
      jit::supports(static_cast<uint32_t>(k), static_cast<uint32_t>(e), sb))
    return net_name("reconstruct", k, e);
  if (decode_kind(k, m, flags_none(), e, have, sb) != 0 && direct_net_async(e, k, sb, mode, k, m, flags_none()))
    return net_name("reconstruct", k, e);
  if (syndrome_pick(k, m, e, flags_none(), sb, mode)) {
    thread_local std::string name;
    name = std::string("syndrome+") +
           (fft_enabled() && fftnet::supports(k, m, sb) ? net_name("fft_encode", k, m) : choose_encode(k, m, sb, 4).name) +
           "+";
    if (jit::enabled() && jit::supports_async(static_cast<uint32_t>(e), static_cast<uint32_t>(e), sb))
      name += net_name("syndrome", e, e);
    else
      name += e <= kMatrixMaxOut ? choose_decode_matrix(static_cast<uint32_t>(e), sb, 4).name
                                 : choose_decode_mtile(static_cast<uint32_t>(e), sb, 4).name;
    return name.c_str();
  }
  switch (decode_kind(k, m, flags_none(), e, have, sb)) {
    case 1: return choose_decode_matrix(static_cast<uint32_t>(e), sb, 4).name;
    case 2: return choose_decode_mtile(static_cast<uint32_t>(e), sb, 4).name;
    default: return choose_decode(k, m, sb, 4).name;
  }
}

int rs_jit_stats(uint64_t *compiles, uint64_t *cache_hits, uint64_t *modules) {
  return guarded([&]() -> int {
    jit::compile_stats(compiles, cache_hits, modules);
    return RS_OK;
  });
}

int rs_net_wait(void) {
  return guarded([&]() -> int {
    jit::wait_pending();
    return RS_OK;
  });
}

int rs_psyn_compile_check(uint64_t k, uint64_t m, uint32_t flags, double *compile_ms, uint64_t *code_bytes) {
  return guarded([&]() -> int {
    int st = check_codec(k, m, jit::kUnitBytes);
    if (st) return st;
    if (is_low_rate(k, m) || (flags & RS_FLAG_QUIRK_D1))
      return fail(RS_ERR_INVALID_ARGUMENT, "no per-stripe syndrome network for this code");
    if (!psyn::supports(k, m, jit::kUnitBytes)) {
      if (!fftnet::supports(k, m, jit::kUnitBytes))
        return fail(RS_ERR_INVALID_ARGUMENT, "no per-stripe syndrome network for this code");
      // wide code: the FFT syndrome kernel with per-stripe masks + the generic solve
      fftnet::Spec fs;
      fs.k = static_cast<uint32_t>(k);
      fs.m = static_cast<uint32_t>(m);
      fs.flags = flags & RS_FLAG_QUIRK_D2;
      fs.dyn = true;
      std::string err;
      size_t b1 = 0, b2 = 0;
      double t1 = 0, t2 = 0;
      if (!fftnet::compile_check(fs, err, &t1, &b1)) return fail(RS_ERR_DEVICE, err);
      if (!psyn::compile_check_solve(cantor_basis(), err, &t2, &b2)) return fail(RS_ERR_DEVICE, err);
      if (compile_ms) *compile_ms = t1 + t2;
      if (code_bytes) *code_bytes = b1 + b2;
      return RS_OK;
    }
    jit::NetSpec map;
    encode_map(k, m, flags & RS_FLAG_QUIRK_D2, map);
    psyn::Spec spec;
    spec.k = static_cast<uint32_t>(k);
    spec.m = static_cast<uint32_t>(m);
    spec.flags = flags & RS_FLAG_QUIRK_D2;
    spec.images = std::move(map.images);
    spec.cantor.assign(cantor_basis(), cantor_basis() + 16);
    std::string err;
    size_t bytes = 0;
    if (!psyn::compile_check(spec, err, compile_ms, &bytes)) return fail(RS_ERR_DEVICE, err);
    if (code_bytes) *code_bytes = bytes;
    return RS_OK;
  });
}

// RS_AMD_FFT_CHECK_INVERSE=1: the checks below take the inverse form (k == m == chunk)
static bool check_inverse(uint64_t k, uint64_t m) {
  const char *e = std::getenv("RS_AMD_FFT_CHECK_INVERSE");
  return e && std::strcmp(e, "1") == 0 && fftnet::supports_inverse(k, m, fftnet::kUnitBytes);
}

int rs_fft_compile_check(uint64_t k, uint64_t m, uint32_t flags, double *compile_ms, uint64_t *code_bytes,
                         uint64_t *valu_ops) {
  return guarded([&]() -> int {
    int st = check_codec(k, m, fftnet::kUnitBytes);
    if (st) return st;
    if (!fftnet::supports(k, m, fftnet::kUnitBytes)) return fail(RS_ERR_INVALID_ARGUMENT, "no FFT kernel form");
    fftnet::Spec spec;
    spec.k = static_cast<uint32_t>(k);
    spec.m = static_cast<uint32_t>(m);
    spec.flags = flags;
    // RS_AMD_FFT_CHECK_PIECES=2: the 1 KiB-shard variant (units of two stripes)
    if (const char *pc = std::getenv("RS_AMD_FFT_CHECK_PIECES")) spec.pieces = std::strcmp(pc, "2") == 0 ? 2 : 1;
    spec.inverse = check_inverse(k, m);
    if (valu_ops) {
      const fftnet::Stats s = fftnet::stats(spec);
      *valu_ops = s.ops_a + s.ops_b + s.ops_io;
    }
    std::string err;
    size_t bytes = 0;
    if (!fftnet::compile_check(spec, err, compile_ms, &bytes)) return fail(RS_ERR_DEVICE, err);
    if (code_bytes) *code_bytes = bytes;
    return RS_OK;
  });
}

int rs_fft_selftest(uint64_t k, uint64_t m, uint32_t flags, const uint8_t *skip, int trials, uint64_t *mismatches) {
  return guarded([&]() -> int {
    int st = check_codec(k, m, fftnet::kUnitBytes);
    if (st) return st;
    if (!fftnet::supports(k, m, fftnet::kUnitBytes)) return fail(RS_ERR_INVALID_ARGUMENT, "no FFT kernel form");
    fftnet::Spec spec;
    spec.k = static_cast<uint32_t>(k);
    spec.m = static_cast<uint32_t>(m);
    spec.flags = flags;
    if (skip) spec.skip.assign(skip, skip + k);
    spec.inverse = check_inverse(k, m);
    const uint64_t bad = fftnet::selftest(spec, trials);
    if (mismatches) *mismatches = bad;
    return RS_OK;
  });
}

int rs_net_compile_check(uint64_t k, uint64_t m, const uint8_t *present, uint32_t flags, double *compile_ms) {
  return guarded([&]() -> int {
    int st = check_codec(k, m, jit::kUnitBytes);
    if (st) return st;
    jit::NetSpec spec;
    if (present) {
      uint64_t have = 0;
      for (uint64_t i = 0; i < k + m; i++) have += present[i] != 0;
      if (have < k) return fail(RS_ERR_NOT_ENOUGH_SHARDS, "fewer than original_count shards present");
      uint64_t e = 0;
      for (uint64_t i = 0; i < k; i++) e += present[i] ? 0 : 1;
      if (is_low_rate(k, m)) {
        if ((st = low_decode_map(k, m, flags, present, spec))) return st;
      } else if (!jit::supports_async(static_cast<uint32_t>(k), static_cast<uint32_t>(e), jit::kUnitBytes) &&
                 syndrome_pick(k, m, e, flags, jit::kUnitBytes * 64, "auto")) {
        if ((st = syndrome_map(k, m, present, spec))) return st;  // the plan's e x e map
      } else {
        reconstruct_map(k, m, flags, present, spec);
      }
    } else if (is_low_rate(k, m)) {
      encode_low_map(k, m, flags, spec);
    } else {
      encode_map(k, m, flags, spec);
    }
    if (!jit::supports_async(spec.n_in, spec.n_out, jit::kUnitBytes))  // also the background-compiled sizes
      return fail(RS_ERR_INVALID_ARGUMENT, "no network form");
    std::string err;
    if (!jit::compile_check(spec, err, compile_ms, nullptr)) return fail(RS_ERR_DEVICE, err);
    return RS_OK;
  });
}

int rs_encode_batch_dev(uint64_t k, uint64_t m, size_t sb, uint64_t n_stripes, const void *d_original,
                        uint64_t orig_stride, void *d_recovery, uint64_t rec_stride, uint32_t flags,
                        rs_stream_t stream) {
  return guarded([&]() -> int {
    if (k == 0) return fail(RS_ERR_TOO_FEW_ORIGINAL_SHARDS, "original_count == 0");
    int st = check_codec(k, m, sb);
    if (st) return st;
    if (n_stripes == 0) return RS_OK;
    if (!d_original || !d_recovery) return fail(RS_ERR_INVALID_ARGUMENT, "NULL device pointer");
    if (orig_stride == 0) orig_stride = k * sb;
    if (rec_stride == 0) rec_stride = m * sb;
    if (sb % 64) {
      int dev;
      if ((st = current_device(&dev))) return st;
      return encode_tail(k, m, sb, n_stripes, static_cast<const uint8_t *>(d_original), orig_stride,
                         static_cast<uint8_t *>(d_recovery), rec_stride, flags, static_cast<hipStream_t>(stream));
    }
    if (orig_stride < k * sb || rec_stride < m * sb) return fail(RS_ERR_INVALID_ARGUMENT, "stripe stride too small");
    const int max_nv = align_nv({reinterpret_cast<uint64_t>(d_original), reinterpret_cast<uint64_t>(d_recovery),
                                 orig_stride, rec_stride});
    if (!max_nv) return fail(RS_ERR_INVALID_ARGUMENT, "device pointers/strides must be 4-byte aligned");
    int dev;
    if ((st = current_device(&dev))) return st;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (is_low_rate(k, m)) {
      std::shared_ptr<MapPlan> lp;
      if ((st = get_low_encode_plan(dev, k, m, flags, lp))) return st;
      return run_map(*lp, sb, n_stripes, static_cast<const uint8_t *>(d_original), orig_stride, nullptr, 0,
                     static_cast<uint8_t *>(d_recovery), rec_stride, max_nv, s);
    }
    std::shared_ptr<EncodePlan> plan;
    if ((st = get_encode_plan(dev, k, m, flags, plan))) return st;
    if (max_nv == 4 && plan->fft && fft_enabled() && fftnet::supports(k, m, sb)) {
      const fftnet::Spec *fs = nullptr;
      if (const jit::Kernel *fk = fft_kernel(*plan->fft, sb, &fs)) {
        HIP_TRY(fftnet::launch(*fk, *fs, static_cast<const uint8_t *>(d_original), orig_stride, nullptr, 0,
                               static_cast<uint8_t *>(d_recovery), rec_stride, sb, n_stripes, s));
        return RS_OK;
      }
    }
    if (max_nv == 4 && jit::enabled() && plan->net->spec.n_in && encode_net_ok(sb) &&
        (plan->net->async ? jit::supports_async(static_cast<uint32_t>(k), static_cast<uint32_t>(m), sb) &&
                                jit::net_pieces(sb) == 1
                          : jit::supports(static_cast<uint32_t>(k), static_cast<uint32_t>(m), sb))) {
      if (const jit::Kernel *nk = net_kernel(*plan->net, sb)) {
        HIP_TRY(jit::launch(*nk, static_cast<const uint8_t *>(d_original), orig_stride, nullptr, 0,
                            static_cast<uint8_t *>(d_recovery), rec_stride, sb, n_stripes, s));
        return RS_OK;
      }
    }
    const KernelChoice kc = choose_encode(k, m, sb, max_nv);
    EncodeArgs a{};
    a.data = static_cast<const uint8_t *>(d_original);
    a.data_stripe_stride = orig_stride;
    a.parity = static_cast<uint8_t *>(d_recovery);
    a.parity_stripe_stride = rec_stride;
    a.shard_bytes = sb;
    a.tabs = static_cast<const RsTab *>(plan->buf->p);
    a.chunk = plan->chunk;
    a.n_chunks = plan->n_chunks;
    a.trunc_first = plan->trunc_first;
    a.trunc_last = plan->trunc_last;
    a.m = static_cast<uint32_t>(m);
    a.k = static_cast<uint32_t>(k);
    a.tabs_per_chunk = plan->tabs_per_chunk;
    a.work = plan->work;
    a.contig = kc.variant != Variant::kGeneric && contig_ok(sb, kc.nv);
    if (kc.variant != Variant::kGeneric) {
      a.n_stripes = n_stripes;
      HIP_TRY(launch_encode(kc, a, s));
      return RS_OK;
    }
    const uint64_t per = std::max<uint64_t>(1, std::min<uint64_t>(n_stripes, kScratchCap / (plan->work * sb)));
    void *scratch = nullptr;
    HIP_TRY(hipMallocAsync(&scratch, per * plan->work * sb, s));
    for (uint64_t s0 = 0; s0 < n_stripes; s0 += per) {
      EncodeArgs b = a;
      b.data += s0 * orig_stride;
      b.parity += s0 * rec_stride;
      b.n_stripes = std::min(per, n_stripes - s0);
      b.scratch = static_cast<uint8_t *>(scratch);
      b.scratch_stripes = per;
      hipError_t e = launch_encode(kc, b, s);
      if (e != hipSuccess) {
        (void)hipFreeAsync(scratch, s);
        return hip_fail(e, "launch_encode");
      }
    }
    HIP_TRY(hipFreeAsync(scratch, s));
    return RS_OK;
  });
}

int rs_reconstruct_batch_dev(uint64_t k, uint64_t m, size_t sb, uint64_t n_stripes, const uint8_t *present,
                             const void *d_original, uint64_t orig_stride, const void *d_recovery,
                             uint64_t rec_stride, void *d_restored, uint64_t out_stride, uint32_t flags,
                             rs_stream_t stream) {
  return guarded([&]() -> int {
    if (!present) return fail(RS_ERR_INVALID_ARGUMENT, "present == NULL");
    int st = check_codec(k, m, sb);
    if (st) return st;
    uint64_t have = 0, e = 0, have_rec = 0;
    for (uint64_t i = 0; i < k; i++) {
      have += present[i] != 0;
      e += present[i] == 0;
    }
    for (uint64_t i = 0; i < m; i++) have_rec += present[k + i] != 0;
    if (have + have_rec < k) return fail(RS_ERR_NOT_ENOUGH_SHARDS, "fewer than original_count shards present");
    if (e == 0 || n_stripes == 0) return RS_OK;  // nothing missing: root.zig:48-57 copy-through
    if (orig_stride == 0) orig_stride = k * sb;
    if (rec_stride == 0) rec_stride = m * sb;
    if (out_stride == 0) out_stride = e * sb;
    if ((have && !d_original) || (have_rec && !d_recovery) || !d_restored)
      return fail(RS_ERR_INVALID_ARGUMENT, "NULL device pointer");
    if (sb % 64) {
      int dev;
      if ((st = current_device(&dev))) return st;
      return reconstruct_tail(k, m, sb, n_stripes, present, e, static_cast<const uint8_t *>(d_original), orig_stride,
                              static_cast<const uint8_t *>(d_recovery), rec_stride, static_cast<uint8_t *>(d_restored),
                              out_stride, flags, static_cast<hipStream_t>(stream));
    }
    const int max_nv =
        align_nv({reinterpret_cast<uint64_t>(d_original), reinterpret_cast<uint64_t>(d_recovery),
                  reinterpret_cast<uint64_t>(d_restored), orig_stride, rec_stride, out_stride});
    if (!max_nv) return fail(RS_ERR_INVALID_ARGUMENT, "device pointers/strides must be 4-byte aligned");
    int dev;
    if ((st = current_device(&dev))) return st;
    if (is_low_rate(k, m)) {
      std::shared_ptr<MapPlan> lp;
      if ((st = get_low_decode_plan(dev, k, m, flags, present, lp))) return st;
      return run_map(*lp, sb, n_stripes, static_cast<const uint8_t *>(d_original), orig_stride,
                     static_cast<const uint8_t *>(d_recovery), rec_stride, static_cast<uint8_t *>(d_restored), out_stride,
                     max_nv, static_cast<hipStream_t>(stream));
    }
    std::shared_ptr<DecodePlan> plan;
    if ((st = get_decode_plan(dev, k, m, sb, flags, present, plan))) return st;
    if (plan->inv_fft && max_nv == 4) {
      const fftnet::Spec *fs = nullptr;
      if (const jit::Kernel *fk = fft_kernel(*plan->inv_fft, sb, &fs)) {
        HIP_TRY(fftnet::launch(*fk, *fs, static_cast<const uint8_t *>(d_recovery), rec_stride, nullptr, 0,
                               static_cast<uint8_t *>(d_restored), out_stride, sb, n_stripes,
                               static_cast<hipStream_t>(stream)));
        return RS_OK;
      }
    }
    if (plan->net && !plan->syndrome && max_nv == 4) {
      if (const jit::Kernel *nk = net_kernel(*plan->net, sb)) {
        HIP_TRY(jit::launch(*nk, static_cast<const uint8_t *>(d_original), orig_stride,
                            static_cast<const uint8_t *>(d_recovery), rec_stride, static_cast<uint8_t *>(d_restored),
                            out_stride, sb, n_stripes, static_cast<hipStream_t>(stream)));
        return RS_OK;
      }
    }
    const KernelChoice kc = plan->tiled    ? choose_decode_mtile(plan->e, sb, max_nv)
                            : plan->matrix ? choose_decode_matrix(plan->e, sb, max_nv)
                                           : choose_decode(k, m, sb, max_nv);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const uint8_t *base = static_cast<const uint8_t *>(plan->buf->p);
    DecodeArgs a{};
    a.orig = static_cast<const uint8_t *>(d_original);
    a.orig_stripe_stride = orig_stride;
    a.rec = static_cast<const uint8_t *>(d_recovery);
    a.rec_stripe_stride = rec_stride;
    a.out = static_cast<uint8_t *>(d_restored);
    a.out_stripe_stride = out_stride;
    a.shard_bytes = sb;
    a.tab_ifft = reinterpret_cast<const RsTab *>(base);
    a.tab_fft = reinterpret_cast<const RsTab *>(base + plan->off_fft);
    a.tab_pre = reinterpret_cast<const RsTab *>(base + plan->off_pre);
    a.tab_post = reinterpret_cast<const RsTab *>(base + plan->off_post);
    a.pos_src = reinterpret_cast<const int32_t *>(base + plan->off_src);
    a.pos_dst = reinterpret_cast<const int32_t *>(base + plan->off_dst);
    a.work = plan->work;
    a.trunc = plan->trunc;
    a.tab_mat = reinterpret_cast<const RsTab *>(base + plan->off_mat);
    a.n_in = plan->n_in;
    a.n_out = plan->e;
    a.contig = kc.variant != Variant::kGeneric && contig_ok(sb, kc.nv);
    if (!a.orig) a.orig = a.rec;  // never dereferenced for absent shards
    if (!a.rec) a.rec = a.orig;
    if (plan->syndrome) {
      // 1) Enc(d') of the received data (erased shards skipped) into a scratch,
      // 2) the e x e matrix kernel on the syndromes rec[R_i] ^ scratch[R_i]
      std::shared_ptr<EncodePlan> ep;
      if ((st = get_encode_plan(dev, k, m, RS_FLAG_CORRECTED, ep))) return st;
      const KernelChoice ke = choose_encode(k, m, sb, max_nv);
      EncodeArgs ea{};
      ea.data = a.orig;
      ea.data_stripe_stride = orig_stride;
      ea.parity_stripe_stride = m * sb;
      ea.shard_bytes = sb;
      ea.tabs = static_cast<const RsTab *>(ep->buf->p);
      ea.chunk = ep->chunk;
      ea.n_chunks = ep->n_chunks;
      ea.trunc_first = ep->trunc_first;
      ea.trunc_last = ep->trunc_last;
      ea.m = static_cast<uint32_t>(m);
      ea.k = static_cast<uint32_t>(k);
      ea.tabs_per_chunk = ep->tabs_per_chunk;
      ea.work = ep->work;
      ea.contig = contig_ok(sb, ke.nv);
      ea.skip = static_cast<const uint32_t *>(plan->skip->p);
      const jit::Kernel *nk = plan->net && max_nv == 4 ? net_kernel(*plan->net, sb) : nullptr;
      // scratch per slice (RS_AMD_SYN_SLICE_MB, default 4096): a slice whose syndromes fit
      // the 256 MB Infinity Cache is read back by the map from there
      const char *sl = std::getenv("RS_AMD_SYN_SLICE_MB");
      const uint64_t cap = (sl && *sl ? std::max(1, std::atoi(sl)) : 4096) * (1ull << 20);
      const uint64_t per = std::max<uint64_t>(1, std::min<uint64_t>(n_stripes, cap / (m * sb)));
      void *scratch = nullptr;
      HIP_TRY(hipMallocAsync(&scratch, per * m * sb, s));
      for (uint64_t s0 = 0; s0 < n_stripes; s0 += per) {
        const uint64_t cnt = std::min(per, n_stripes - s0);
        EncodeArgs eb = ea;
        eb.data += s0 * orig_stride;
        eb.parity = static_cast<uint8_t *>(scratch);
        eb.n_stripes = cnt;
        DecodeArgs db = a;
        db.orig += s0 * orig_stride;
        db.rec += s0 * rec_stride;
        db.out += s0 * out_stride;
        db.xsrc = static_cast<const uint8_t *>(scratch);
        db.xsrc_stripe_stride = m * sb;
        db.n_stripes = cnt;
        hipError_t err = hipSuccess;
        const fftnet::Spec *fs = nullptr;
        const jit::Kernel *fk = plan->syn_fft && max_nv == 4 ? fft_kernel(*plan->syn_fft, sb, &fs) : nullptr;
        if (fk)
          err = fftnet::launch(*fk, *fs, eb.data, orig_stride, nullptr, 0, eb.parity, m * sb, sb, cnt, s);
        else
          err = launch_encode(ke, eb, s);
        if (err == hipSuccess) {
          if (nk)
            err = jit::launch(*nk, db.orig, orig_stride, db.rec, rec_stride, db.out, out_stride, sb, cnt, s, db.xsrc,
                              db.xsrc_stripe_stride);
          else
            err = launch_decode(kc, db, s);
        }
        if (err != hipSuccess) {
          (void)hipFreeAsync(scratch, s);
          return hip_fail(err, "syndrome reconstruct");
        }
      }
      HIP_TRY(hipFreeAsync(scratch, s));
      return RS_OK;
    }
    if (kc.variant != Variant::kGeneric) {
      a.n_stripes = n_stripes;
      HIP_TRY(launch_decode(kc, a, s));
      return RS_OK;
    }
    const uint64_t per = std::max<uint64_t>(1, std::min<uint64_t>(n_stripes, kScratchCap / (plan->work * sb)));
    void *scratch = nullptr;
    HIP_TRY(hipMallocAsync(&scratch, per * plan->work * sb, s));
    for (uint64_t s0 = 0; s0 < n_stripes; s0 += per) {
      DecodeArgs b = a;
      b.orig += s0 * orig_stride;
      b.rec += s0 * rec_stride;
      b.out += s0 * out_stride;
      b.tab_pre += s0 * a.pattern_stride;
      b.tab_post += s0 * a.pattern_stride;
      b.pos_src += s0 * a.pattern_stride;
      b.pos_dst += s0 * a.pattern_stride;
      b.n_stripes = std::min(per, n_stripes - s0);
      b.scratch = static_cast<uint8_t *>(scratch);
      b.scratch_stripes = per;
      hipError_t err = launch_decode(kc, b, s);
      if (err != hipSuccess) {
        (void)hipFreeAsync(scratch, s);
        return hip_fail(err, "launch_decode");
      }
    }
    HIP_TRY(hipFreeAsync(scratch, s));
    return RS_OK;
  });
}

// ------------------------------------------------ per-stripe erasure patterns
namespace {

struct DeviceTables {  // exp, log, log_walsh in HBM (384 KiB per device)
  std::shared_ptr<DevBuf> buf;
};
std::map<int, DeviceTables> g_dev_tables;

int device_tables(int dev, const uint16_t **exp, const uint16_t **log, const uint16_t **lw) {
  std::lock_guard<std::mutex> lk(g_plan_mu);
  auto it = g_dev_tables.find(dev);
  if (it == g_dev_tables.end()) {
    const Tables &t = tables();
    std::vector<uint16_t> blob(3 * kOrder);
    std::memcpy(blob.data(), t.exp, kOrder * 2);
    std::memcpy(blob.data() + kOrder, t.log, kOrder * 2);
    std::memcpy(blob.data() + 2 * kOrder, t.log_walsh, kOrder * 2);
    DeviceTables d;
    int st = upload(blob.data(), blob.size() * 2, dev, d.buf);
    if (st) return st;
    it = g_dev_tables.emplace(dev, d).first;
  }
  const uint16_t *b = static_cast<const uint16_t *>(it->second.buf->p);
  *exp = b;
  *log = b + kOrder;
  *lw = b + 2 * kOrder;
  return RS_OK;
}

std::map<std::string, std::shared_ptr<DevBuf>> g_twiddle_plans;  // IFFT+FFT tables of size W, skew_delta 0

int twiddle_plan(int dev, uint64_t W, uint32_t flags, std::shared_ptr<DevBuf> &out, size_t &off_fft) {
  const bool d1 = flags & RS_FLAG_QUIRK_D1;
  std::vector<RsTab> tabs;
  push_ifft_tabs(tabs, W, 0, d1);
  off_fft = tabs.size() * sizeof(RsTab);
  const std::string key = std::to_string(dev) + "/" + std::to_string(W) + "/" + std::to_string(d1);
  std::lock_guard<std::mutex> lk(g_plan_mu);
  auto it = g_twiddle_plans.find(key);
  if (it != g_twiddle_plans.end()) {
    out = it->second;
    return RS_OK;
  }
  push_fft_tabs(tabs, W, 0, d1);
  int st = upload(tabs.data(), tabs.size() * sizeof(RsTab), dev, out);
  if (st) return st;
  g_twiddle_plans.emplace(key, out);
  return RS_OK;
}

// Per code (k, m, flags): the syndrome-network kernel of rs_psyn.hpp and the code's
// encode coefficients G [m][k] in HBM (for the per-stripe plans).
struct PsynPlan {
  std::mutex mu;
  bool failed = false;
  psyn::Spec spec;
  std::shared_ptr<DevBuf> G;
};
std::map<std::string, std::shared_ptr<PsynPlan>> g_psyn_plans;

int psyn_plan(int dev, uint64_t k, uint64_t m, uint32_t flags, std::shared_ptr<PsynPlan> &out) {
  const std::string key = std::to_string(dev) + "/" + std::to_string(k) + "/" + std::to_string(m) + "/" +
                          std::to_string(flags & RS_FLAG_QUIRK_D2);
  {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    auto it = g_psyn_plans.find(key);
    if (it != g_psyn_plans.end()) {
      out = it->second;
      return RS_OK;
    }
  }
  auto p = std::make_shared<PsynPlan>();
  jit::NetSpec map;
  encode_map(k, m, flags & RS_FLAG_QUIRK_D2, map);
  std::vector<uint16_t> G(m * k + 16);  // coefficients, then the Cantor basis (launch_psyn_plan)
  for (uint64_t t = 0; t < k; t++)
    for (uint64_t r = 0; r < m; r++) G[r * k + t] = map.images[(t * m + r) * 16];  // image of 1 = the coefficient
  std::copy(cantor_basis(), cantor_basis() + 16, G.begin() + m * k);
  p->spec.cantor.assign(cantor_basis(), cantor_basis() + 16);
  int st = upload(G.data(), G.size() * sizeof(uint16_t), dev, p->G);
  if (st) return st;
  p->spec.k = static_cast<uint32_t>(k);
  p->spec.m = static_cast<uint32_t>(m);
  p->spec.flags = flags & RS_FLAG_QUIRK_D2;
  p->spec.images = std::move(map.images);
  std::lock_guard<std::mutex> lk(g_plan_mu);
  out = g_psyn_plans.emplace(key, p).first->second;
  return RS_OK;
}

const jit::Kernel *psyn_kernel(PsynPlan &p) {
  std::lock_guard<std::mutex> lk(p.mu);
  if (p.failed) return nullptr;
  std::string err;
  const jit::Kernel *k = psyn::get(p.spec, err);
  if (!k) {
    p.failed = true;
    warn_once_per_reason("[rs_amd] per-stripe syndrome network unavailable, using table kernels: ", err);
  }
  return k;
}

// Wide codes: the FFT kernel with per-stripe masks for the syndromes + the generic solve
struct WpsSlot {
  std::shared_ptr<FftSlot> fft = std::make_shared<FftSlot>();
  std::mutex mu;
  bool solve_failed = false;
};
std::map<std::string, std::shared_ptr<WpsSlot>> g_wps;

void wps_slot(int dev, uint64_t k, uint64_t m, uint32_t flags, std::shared_ptr<WpsSlot> &out) {
  const std::string key = std::to_string(dev) + "/" + std::to_string(k) + "/" + std::to_string(m) + "/" +
                          std::to_string(flags & RS_FLAG_QUIRK_D2);
  std::lock_guard<std::mutex> lk(g_plan_mu);
  auto &p = g_wps[key];
  if (!p) {
    p = std::make_shared<WpsSlot>();
    fftnet::Spec &fs = p->fft->spec;
    fs.k = static_cast<uint32_t>(k);
    fs.m = static_cast<uint32_t>(m);
    fs.flags = flags & RS_FLAG_QUIRK_D2;
    fs.dyn = true;
  }
  out = p;
}

// Under D2 a code with k > chunk and k % chunk == 0 drops its last full chunk
// (root.zig:151): the encode ignores those shards, the code is not MDS, and the
// per-stripe e x e solves can be singular. Such codes take the FFT kernels, which
// follow root.zig:268-335 as written.
bool d2_drops_chunk(uint64_t k, uint64_t m, uint32_t flags) {
  const uint64_t C = ceil_pow2(m);
  return (flags & RS_FLAG_QUIRK_D2) && k > C && k % C == 0;
}

bool wps_enabled(uint64_t k, uint64_t m, uint64_t sb, uint32_t flags, uint32_t max_e) {
  const char *pm = std::getenv("RS_AMD_PATTERNS");
  const std::string mode = pm ? pm : "";
  return !(flags & RS_FLAG_QUIRK_D1) && !d2_drops_chunk(k, m, flags) &&
         (mode.empty() || mode == "auto" || mode == "psyn") && fft_enabled() && fftnet::supports(k, m, sb) && fftnet::pieces(sb) == 1 && sb % jit::kUnitBytes == 0 &&
         m <= 64;  // max_e up to m: output groups of 8 (rs_psyn.hpp launch_solve)
}

bool psyn_enabled(uint64_t k, uint64_t m, uint64_t sb, uint32_t flags) {
  const char *pm = std::getenv("RS_AMD_PATTERNS");
  const std::string mode = pm ? pm : "";
  return !(flags & RS_FLAG_QUIRK_D1) && !d2_drops_chunk(k, m, flags) &&
         (mode.empty() || mode == "auto" || mode == "psyn") && jit::enabled() && psyn::supports(k, m, sb);
}

}  // namespace

const char *rs_patterns_kernel_name(uint64_t k, uint64_t m, size_t sb, uint32_t max_e, uint32_t flags) {
  thread_local std::string name;
  if (psyn_enabled(k, m, sb, flags)) {
    name = "psyn_k" + std::to_string(k) + "_m" + std::to_string(m);
  } else if (wps_enabled(k, m, sb, flags, max_e)) {
    name = "fft_syndromes+psyn_solve";
  } else {
    const char *pm = std::getenv("RS_AMD_PATTERNS");
    const uint64_t W = ceil_pow2(ceil_pow2(m) + k);
    const bool matrix =
        !(flags & RS_FLAG_QUIRK_D1) && W <= 32 && max_e <= kMatrixMaxOut && !(pm && std::string(pm) == "fft");
    name = matrix ? "pattern_matrix" : "pattern_fft";
  }
  return name.c_str();
}

int rs_reconstruct_batch_dev_patterns(uint64_t k, uint64_t m, size_t sb, uint64_t n_stripes, const uint8_t *d_present,
                                      uint64_t present_stride, uint32_t max_e, const void *d_original,
                                      uint64_t orig_stride, const void *d_recovery, uint64_t rec_stride,
                                      void *d_restored, uint64_t out_stride, int32_t *d_status, uint32_t flags,
                                      rs_stream_t stream) {
  return guarded([&]() -> int {
    int st = check_codec(k, m, sb);
    if (st == RS_OK && is_low_rate(k, m))
      return fail(RS_ERR_LOW_RATE_UNSUPPORTED, "per-stripe patterns: high-rate codes only");
    if (st) return st;
    if (n_stripes == 0 || max_e == 0) return RS_OK;
    if (!d_present || !d_original || !d_recovery || !d_restored) return fail(RS_ERR_INVALID_ARGUMENT, "NULL pointer");
    if (sb % 64) return fail(RS_ERR_SHARD_TAIL_UNSUPPORTED, "per-stripe patterns need shard_bytes % 64 == 0");
    if (present_stride == 0) present_stride = k + m;
    if (orig_stride == 0) orig_stride = k * sb;
    if (rec_stride == 0) rec_stride = m * sb;
    if (out_stride == 0) out_stride = static_cast<uint64_t>(max_e) * sb;
    const int max_nv = align_nv({reinterpret_cast<uint64_t>(d_original), reinterpret_cast<uint64_t>(d_recovery),
                                 reinterpret_cast<uint64_t>(d_restored), orig_stride, rec_stride, out_stride});
    if (!max_nv) return fail(RS_ERR_INVALID_ARGUMENT, "device pointers/strides must be 4-byte aligned");
    int dev;
    if ((st = current_device(&dev))) return st;
    const uint64_t C = ceil_pow2(m), W = ceil_pow2(C + k);
    const uint16_t *dexp, *dlog, *dlw;
    if ((st = device_tables(dev, &dexp, &dlog, &dlw))) return st;
    // syndrome network (rs_psyn.hpp): the code's fixed k -> m network plus a per-stripe
    // e x e solve; corrected multiply, k <= 64, m <= 4, whole 4 KiB units
    if (max_nv == 4 && psyn_enabled(k, m, sb, flags)) {
      std::shared_ptr<PsynPlan> pp;
      if ((st = psyn_plan(dev, k, m, flags, pp))) return st;
      if (const jit::Kernel *pk = psyn_kernel(*pp)) {
        hipStream_t s = static_cast<hipStream_t>(stream);
        const uint32_t mo = psyn::max_out(static_cast<uint32_t>(k), static_cast<uint32_t>(m));
        const uint32_t pdw = psyn::plan_dwords(static_cast<uint32_t>(k), static_cast<uint32_t>(m));
        void *blk = nullptr;
        HIP_TRY(hipMallocAsync(&blk, n_stripes * pdw * sizeof(uint32_t), s));
        hipError_t e = launch_psyn_plan(d_present, present_stride, static_cast<uint32_t>(k), static_cast<uint32_t>(m), mo,
                                        max_e, n_stripes, static_cast<const uint16_t *>(pp->G->p), dexp, dlog,
                                        static_cast<uint32_t *>(blk), pdw, d_status, s);
        if (e == hipSuccess)
          e = psyn::launch(*pk, pp->spec, static_cast<const uint8_t *>(d_original), orig_stride,
                           static_cast<const uint8_t *>(d_recovery), rec_stride, static_cast<uint8_t *>(d_restored),
                           out_stride, sb, n_stripes, static_cast<const uint32_t *>(blk), s);
        (void)hipFreeAsync(blk, s);
        if (e != hipSuccess) return hip_fail(e, "per-stripe syndrome network");
        return RS_OK;
      }
    }
    // wide codes: syndromes on the FFT kernel (per-stripe masks), then the e x e solve
    if (max_nv == 4 && wps_enabled(k, m, sb, flags, max_e)) {
      std::shared_ptr<PsynPlan> pp;  // G and the Cantor basis
      if ((st = psyn_plan(dev, k, m, flags, pp))) return st;
      std::shared_ptr<WpsSlot> ws;
      wps_slot(dev, k, m, flags, ws);
      const fftnet::Spec *fs = nullptr;
      const jit::Kernel *fk = fft_kernel(*ws->fft, sb, &fs);
      const jit::Kernel *sk = nullptr;
      {
        std::lock_guard<std::mutex> lk(ws->mu);
        if (!ws->solve_failed) {
          std::string err;
          sk = psyn::get_solve(cantor_basis(), err);
          if (!sk) {
            ws->solve_failed = true;
            warn_once_per_reason("[rs_amd] per-stripe solve kernel unavailable, using table kernels: ", err);
          }
        }
      }
      if (fk && sk) {
        hipStream_t s = static_cast<hipStream_t>(stream);
        // coefficients for min(max_e, m) outputs per syndrome, in groups of 8
        const uint32_t cs = wps_coef_stride(static_cast<uint32_t>(std::min<uint64_t>(max_e, m)));
        const uint32_t dmw = fftnet::dyn_mask_words(*fs), pw = dmw + 2 + 64 + 64 * cs;
        const uint64_t per = std::max<uint64_t>(1, std::min<uint64_t>(n_stripes, kScratchCap / (m * sb)));
        void *blk = nullptr, *scratch = nullptr;
        HIP_TRY(hipMallocAsync(&blk, n_stripes * pw * sizeof(uint32_t), s));
        hipError_t e = hipMallocAsync(&scratch, per * m * sb, s);
        if (e == hipSuccess)
          e = launch_wps_plan(d_present, present_stride, static_cast<uint32_t>(k), static_cast<uint32_t>(m),
                              static_cast<uint32_t>(std::min<uint64_t>(max_e, m)), n_stripes, static_cast<const uint16_t *>(pp->G->p), dexp, dlog, static_cast<uint32_t *>(blk),
                              pw, dmw, d_status, s);
        for (uint64_t s0 = 0; e == hipSuccess && s0 < n_stripes; s0 += per) {
          const uint64_t cnt = std::min(per, n_stripes - s0);
          const uint32_t *bl = static_cast<const uint32_t *>(blk) + s0 * pw;
          e = fftnet::launch(*fk, *fs, static_cast<const uint8_t *>(d_original) + s0 * orig_stride, orig_stride, nullptr,
                             0, static_cast<uint8_t *>(scratch), m * sb, sb, cnt, s, bl, pw);
          if (e == hipSuccess)
            e = psyn::launch_solve(*sk, static_cast<const uint8_t *>(d_recovery) + s0 * rec_stride, rec_stride,
                                   static_cast<const uint8_t *>(scratch), m * sb,
                                   static_cast<uint8_t *>(d_restored) + s0 * out_stride, out_stride, sb, cnt, bl, pw,
                                   dmw, cs, s);
        }
        if (scratch) (void)hipFreeAsync(scratch, s);
        (void)hipFreeAsync(blk, s);
        if (e != hipSuccess) return hip_fail(e, "per-stripe wide-code reconstruct");
        return RS_OK;
      }
    }
    std::shared_ptr<DevBuf> tw;
    size_t off_fft = 0;
    if ((st = twiddle_plan(dev, W, flags, tw, off_fft))) return st;
    hipStream_t s = static_cast<hipStream_t>(stream);
    // matrix path (below): corrected multiply, W <= 32, max_e <= 8
    const char *pm = std::getenv("RS_AMD_PATTERNS");
    const bool use_matrix =
        !(flags & RS_FLAG_QUIRK_D1) && W <= 32 && max_e <= kMatrixMaxOut && !(pm && std::string(pm) == "fft");
    // per-stripe plan: logs u16 | pre RsTab | post RsTab | src i32 | dst i32 (W entries each)
    //                  [| trimmed present rows, matrix path]
    const uint64_t per = W * (2 + 2 * sizeof(RsTab) + 8);
    void *tmp = nullptr;
    HIP_TRY(hipMallocAsync(&tmp, n_stripes * per + (use_matrix ? n_stripes * (k + m) : 0) + 256, s));
    if (use_matrix) {  // evaluate the erasure locator for exactly the k inputs the matrix uses
      uint8_t *trimmed = static_cast<uint8_t *>(tmp) + n_stripes * per;
      hipError_t e = launch_trim_present(d_present, present_stride, static_cast<uint32_t>(k), static_cast<uint32_t>(m),
                                         n_stripes, trimmed, s);
      if (e != hipSuccess) {
        (void)hipFreeAsync(tmp, s);
        return hip_fail(e, "launch_trim_present");
      }
      d_present = trimmed;
      present_stride = k + m;
    }
    uint8_t *base = static_cast<uint8_t *>(tmp);
    RsTab *pre = reinterpret_cast<RsTab *>(base);
    RsTab *post = pre + n_stripes * W;
    int32_t *src = reinterpret_cast<int32_t *>(post + n_stripes * W);
    int32_t *dst = src + n_stripes * W;
    uint16_t *logs = reinterpret_cast<uint16_t *>(dst + n_stripes * W);
    hipError_t e = launch_pattern_plan(d_present, present_stride, static_cast<uint32_t>(k), static_cast<uint32_t>(m),
                                       static_cast<uint32_t>(C), static_cast<uint32_t>(W), n_stripes, max_e,
                                       flags & RS_FLAG_QUIRK_D1, dexp, dlog, dlw, logs, pre, post, src, dst, d_status,
                                       s);
    if (e != hipSuccess) {
      (void)hipFreeAsync(tmp, s);
      return hip_fail(e, "launch_pattern_plan");
    }
    // Per-stripe e x k matrices built on the GPU, then the matrix kernel (40 MACs per
    // column for RS(10,4) instead of the FFT reconstruct's 48 multiplies + masks).
    // Corrected multiply only (under D1 the literal reconstruct uses all received
    // shards); RS_AMD_PATTERNS=fft keeps the FFT kernels.
    if (use_matrix) {
      const uint64_t nk = n_stripes * k;
      void *mt = nullptr;
      const uint64_t img_bytes = nk * max_e * 16 * sizeof(uint16_t), tab_bytes = nk * max_e * sizeof(RsTab);
      e = hipMallocAsync(&mt, tab_bytes + img_bytes + nk * 4 + n_stripes * 4 + 256, s);
      if (e == hipSuccess) {
        RsTab *mtabs = static_cast<RsTab *>(mt);
        uint16_t *images = reinterpret_cast<uint16_t *>(static_cast<uint8_t *>(mt) + tab_bytes);
        int32_t *srcs = reinterpret_cast<int32_t *>(static_cast<uint8_t *>(mt) + tab_bytes + img_bytes);
        int32_t *nout = srcs + nk;
        e = launch_pattern_matrix(d_present, present_stride, static_cast<uint32_t>(k), static_cast<uint32_t>(m),
                                  static_cast<uint32_t>(C), static_cast<uint32_t>(W), n_stripes, max_e, logs,
                                  static_cast<const RsTab *>(tw->p),
                                  reinterpret_cast<const RsTab *>(static_cast<const uint8_t *>(tw->p) + off_fft), dexp,
                                  dlog, images, mtabs, srcs, nout, s);
        if (e == hipSuccess) {
          const KernelChoice km = choose_decode_matrix(max_e, sb, max_nv);
          DecodeArgs a{};
          a.orig = static_cast<const uint8_t *>(d_original);
          a.orig_stripe_stride = orig_stride;
          a.rec = static_cast<const uint8_t *>(d_recovery);
          a.rec_stripe_stride = rec_stride;
          a.out = static_cast<uint8_t *>(d_restored);
          a.out_stripe_stride = out_stride;
          a.shard_bytes = sb;
          a.tab_mat = mtabs;
          a.pos_src = srcs;
          a.n_in = static_cast<uint32_t>(k);
          a.n_out = max_e;
          a.mat_stride = k * max_e;
          a.src_stride = k;
          a.nout = nout;
          a.tab_pre = a.tab_post = mtabs;  // unused; launch_decode advances them
          a.pos_dst = srcs;
          a.contig = contig_ok(sb, km.nv);
          a.n_stripes = n_stripes;
          e = launch_decode(km, a, s);
        }
        (void)hipFreeAsync(mt, s);
      }
      (void)hipFreeAsync(tmp, s);
      if (e != hipSuccess) return hip_fail(e, "per-stripe matrix reconstruct");
      return RS_OK;
    }
    const KernelChoice kc = choose_decode(k, m, sb, max_nv);
    DecodeArgs a{};
    a.orig = static_cast<const uint8_t *>(d_original);
    a.orig_stripe_stride = orig_stride;
    a.rec = static_cast<const uint8_t *>(d_recovery);
    a.rec_stripe_stride = rec_stride;
    a.out = static_cast<uint8_t *>(d_restored);
    a.out_stripe_stride = out_stride;
    a.shard_bytes = sb;
    a.tab_ifft = static_cast<const RsTab *>(tw->p);
    a.tab_fft = reinterpret_cast<const RsTab *>(static_cast<const uint8_t *>(tw->p) + off_fft);
    a.tab_pre = pre;
    a.tab_post = post;
    a.pos_src = src;
    a.pos_dst = dst;
    a.work = static_cast<uint32_t>(W);
    a.trunc = static_cast<uint32_t>(C + k);
    a.pattern_stride = W;
    a.contig = kc.variant != Variant::kGeneric && contig_ok(sb, kc.nv);
    if (kc.variant != Variant::kGeneric) {
      a.n_stripes = n_stripes;
      e = launch_decode(kc, a, s);
    } else {
      const uint64_t cap = std::max<uint64_t>(1, std::min<uint64_t>(n_stripes, kScratchCap / (W * sb)));
      void *scratch = nullptr;
      e = hipMallocAsync(&scratch, cap * W * sb, s);
      for (uint64_t s0 = 0; e == hipSuccess && s0 < n_stripes; s0 += cap) {
        DecodeArgs b = a;
        b.orig += s0 * orig_stride;
        b.rec += s0 * rec_stride;
        b.out += s0 * out_stride;
        b.tab_pre += s0 * W;
        b.tab_post += s0 * W;
        b.pos_src += s0 * W;
        b.pos_dst += s0 * W;
        b.n_stripes = std::min(cap, n_stripes - s0);
        b.scratch = static_cast<uint8_t *>(scratch);
        e = launch_decode(kc, b, s);
      }
      if (scratch) (void)hipFreeAsync(scratch, s);
    }
    (void)hipFreeAsync(tmp, s);
    if (e != hipSuccess) return hip_fail(e, "launch_decode (patterns)");
    return RS_OK;
  });
}

// ------------------------------------------------------- host-resident batch
namespace {

// Copy `rows` rows of `row_bytes` between (possibly strided) buffers.
hipError_t copy_rows(void *dst, uint64_t dst_stride, const void *src, uint64_t src_stride, uint64_t row_bytes,
                     uint64_t rows, hipMemcpyKind kind, hipStream_t s) {
  if (rows == 0 || row_bytes == 0) return hipSuccess;
  if (dst_stride == row_bytes && src_stride == row_bytes)
    return hipMemcpyAsync(dst, src, rows * row_bytes, kind, s);
  return hipMemcpy2DAsync(dst, dst_stride, src, src_stride, row_bytes, rows, kind, s);
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
  int ensure(const uint64_t bytes[3], int want) {
    for (int i = 0; i < want; i++)
      if (!st[i]) HIP_TRY(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    bool grow = want != slots;
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
        if (cap[j]) HIP_TRY(hipMalloc(&buf[i][j], cap[j]));
    slots = want;
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
uint64_t host_slice_bytes() {
  const char *e = std::getenv("RS_AMD_HOST_SLICE_MB");
  return (e && *e ? static_cast<uint64_t>(std::max(1, std::atoi(e))) : 256ull) << 20;
}

// Every slot stream is drained before a host-batch call returns, also after an error:
// no copy into the caller's buffers (or out of them) outlives the call.
int drain_after(Pipeline &p, int rc) {
  const int fin = p.finish();
  return rc ? rc : fin;
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

int rs_encode_batch_host(uint64_t k, uint64_t m, size_t sb, uint64_t n, const void *h_orig, uint64_t orig_stride,
                         void *h_rec, uint64_t rec_stride, uint32_t flags) {
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
    auto slices = [&]() -> int {
      for (uint64_t s0 = 0, i = 0; s0 < n; s0 += S, i++) {
        const int slot = static_cast<int>(i % static_cast<uint64_t>(slots));
        const uint64_t cnt = std::min(S, n - s0);
        hipStream_t q = p.st[slot];
        if (inject_host_failure(i)) return fail(RS_ERR_DEVICE, "injected host-batch failure");
        HIP_TRY(copy_rows(p.buf[slot][0], k * sb, static_cast<const uint8_t *>(h_orig) + s0 * orig_stride,
                          orig_stride, k * sb, cnt, hipMemcpyHostToDevice, q));
        int rc = rs_encode_batch_dev(k, m, sb, cnt, p.buf[slot][0], 0, p.buf[slot][1], 0, flags, q);
        if (rc) return rc;
        HIP_TRY(copy_rows(static_cast<uint8_t *>(h_rec) + s0 * rec_stride, rec_stride, p.buf[slot][1], m * sb,
                          m * sb, cnt, hipMemcpyDeviceToHost, q));
      }
      return RS_OK;
    };
    return drain_after(p, slices());
  });
}

int rs_reconstruct_batch_host(uint64_t k, uint64_t m, size_t sb, uint64_t n, const uint8_t *present,
                              const void *h_orig, uint64_t orig_stride, const void *h_rec, uint64_t rec_stride,
                              void *h_out, uint64_t out_stride, uint32_t flags) {
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
    const uint64_t S = std::max<uint64_t>(1, std::min<uint64_t>(n, host_slice_bytes() / (k * sb)));
    const int slots = host_slots();
    Pipeline &p = Pipelines::of(dev);
    std::lock_guard<std::mutex> lk(p.mu);
    const uint64_t bytes[3] = {S * k * sb, S * m * sb, S * e * sb};
    if ((st = p.ensure(bytes, slots))) return st;
    auto slices = [&]() -> int {
      for (uint64_t s0 = 0, i = 0; s0 < n; s0 += S, i++) {
        const int slot = static_cast<int>(i % static_cast<uint64_t>(slots));
        const uint64_t cnt = std::min(S, n - s0);
        hipStream_t q = p.st[slot];
        if (inject_host_failure(i)) return fail(RS_ERR_DEVICE, "injected host-batch failure");
        // only the present shards cross PCIe
        for (uint64_t j = 0; j < k; j++)
          if (present[j])
            HIP_TRY(copy_rows(static_cast<uint8_t *>(p.buf[slot][0]) + j * sb, k * sb,
                              static_cast<const uint8_t *>(h_orig) + s0 * orig_stride + j * sb, orig_stride, sb, cnt,
                              hipMemcpyHostToDevice, q));
        for (uint64_t j = 0; j < m; j++)
          if (present[k + j])
            HIP_TRY(copy_rows(static_cast<uint8_t *>(p.buf[slot][1]) + j * sb, m * sb,
                              static_cast<const uint8_t *>(h_rec) + s0 * rec_stride + j * sb, rec_stride, sb, cnt,
                              hipMemcpyHostToDevice, q));
        int rc = rs_reconstruct_batch_dev(k, m, sb, cnt, present, p.buf[slot][0], 0, p.buf[slot][1], 0,
                                          p.buf[slot][2], 0, flags, q);
        if (rc) return rc;
        HIP_TRY(copy_rows(static_cast<uint8_t *>(h_out) + s0 * out_stride, out_stride, p.buf[slot][2], e * sb,
                          e * sb, cnt, hipMemcpyDeviceToHost, q));
      }
      return RS_OK;
    };
    return drain_after(p, slices());
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
    hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&c->h), nb, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&c->d), nb);
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

int rs_encode(uint64_t k, uint64_t m, size_t sb, const uint8_t *const *original, uint8_t *const *recovery_out) {
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
  HIP_TRY(hipMalloc(&dt.p, std::max<size_t>(16, tabs.size() * sizeof(RsTab))));
  if (!tabs.empty()) HIP_TRY(hipMemcpy(dt.p, tabs.data(), tabs.size() * sizeof(RsTab), hipMemcpyHostToDevice));
  HIP_TRY(hipMalloc(&dw.p, count * sb));
  HIP_TRY(hipMemcpy(dw.p, shards, count * sb, hipMemcpyHostToDevice));
  HIP_TRY(launch_engine_fft(static_cast<uint8_t *>(dw.p), sb, pos, size, trunc, static_cast<const RsTab *>(dt.p),
                            inverse, nullptr));
  HIP_TRY(hipMemcpy(shards, dw.p, count * sb, hipMemcpyDeviceToHost));
  return RS_OK;
}

int rs_engine_fft(uint8_t *shards, uint64_t count, size_t sb, uint64_t pos, uint64_t size, uint64_t trunc,
                  uint64_t sd, uint32_t flags) {
  return guarded([&]() -> int {
    return engine_transform(shards, count, sb, pos, size, trunc, sd, flags, false);
  });
}

int rs_engine_ifft(uint8_t *shards, uint64_t count, size_t sb, uint64_t pos, uint64_t size, uint64_t trunc,
                   uint64_t sd, uint32_t flags) {
  return guarded([&]() -> int {
    return engine_transform(shards, count, sb, pos, size, trunc, sd, flags, true);
  });
}

int rs_engine_mul_scalar(uint8_t *chunks, size_t bytes, uint16_t log_m, uint32_t flags) {
  return guarded([&]() -> int {
    if (!chunks) return fail(RS_ERR_INVALID_ARGUMENT, "NULL chunks");
    if (bytes == 0 || bytes % 64) return fail(RS_ERR_INVALID_SHARD_SIZE, "bytes must be a multiple of 64");
    int dev, st;
    if ((st = current_device(&dev))) return st;
    const RsTab t = make_tab(log_m, flags & RS_FLAG_QUIRK_D1);
    DevMem dt, dw;
    HIP_TRY(hipMalloc(&dt.p, sizeof t));
    HIP_TRY(hipMemcpy(dt.p, &t, sizeof t, hipMemcpyHostToDevice));
    HIP_TRY(hipMalloc(&dw.p, bytes));
    HIP_TRY(hipMemcpy(dw.p, chunks, bytes, hipMemcpyHostToDevice));
    HIP_TRY(launch_mul_scalar(static_cast<uint8_t *>(dw.p), bytes, static_cast<const RsTab *>(dt.p), nullptr));
    HIP_TRY(hipMemcpy(chunks, dw.p, bytes, hipMemcpyDeviceToHost));
    return RS_OK;
  });
}

int rs_engine_eval_poly(uint16_t *erasures, uint64_t trunc) {
  return guarded([&]() -> int {
    if (!erasures) return fail(RS_ERR_INVALID_ARGUMENT, "NULL erasures");
    if (trunc > kOrder) return fail(RS_ERR_INVALID_ARGUMENT, "truncated_size > 65536");
    eval_poly(erasures, trunc);
    return RS_OK;
  });
}

}  // extern "C"
