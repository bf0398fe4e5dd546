// rs_patterns.cpp — rs_reconstruct_batch_dev_patterns: one erasure pattern per stripe
// (§8 f2), the erasure locator and per-stripe plans built on the GPU.
#include "rs_host.hpp"

#include <unordered_map>

using namespace rs;
using namespace rs::host;

namespace rs {
namespace host {
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
    fftnet::Spec &ds = p->dec->spec;
    ds.k = static_cast<uint32_t>(k);
    ds.m = static_cast<uint32_t>(m);
    ds.dyn = ds.decode = true;
    p->decb->spec = ds;
    p->decb->spec.blocked = true;
  }
  out = p;
}

int fdec_mode() {
  const char *e = std::getenv("RS_AMD_FDEC");
  if (e && std::strcmp(e, "0") == 0) return 0;
  if (e && std::strcmp(e, "1") == 0) return 1;
  return 2;
}

bool pdec_enabled() {
  const char *e = std::getenv("RS_AMD_PDEC");
  return fdec_mode() != 1 && !(e && std::strcmp(e, "0") == 0);
}

namespace {
int env_num(const char *name, int def, int lo) {
  const char *e = std::getenv(name);
  return e && *e ? std::max(lo, std::atoi(e)) : def;
}
}  // namespace

uint32_t pdec_after() { return static_cast<uint32_t>(env_num("RS_AMD_PDEC_AFTER", 2, 1)); }
size_t pdec_queue() { return static_cast<size_t>(env_num("RS_AMD_PDEC_QUEUE", 2, 0)); }

bool pdec_admit(int dev, uint64_t k, uint64_t m, const std::string &key) {
  static std::mutex mu;
  static std::map<std::string, std::set<std::string>> admitted;  // code -> pattern keys
  const size_t cap = static_cast<size_t>(env_num("RS_AMD_PDEC_MAX", 32, 0));
  const std::string code = std::to_string(dev) + "/" + std::to_string(k) + "/" + std::to_string(m);
  std::lock_guard<std::mutex> lk(mu);
  std::set<std::string> &s = admitted[code];
  if (s.count(key)) return true;
  if (s.size() >= cap) return false;
  s.insert(key);
  return true;
}

// corrected multiply only (under D1 the literal decode is no inverse of the encode), and
// no code whose D2 encode drops a chunk (its parity is no codeword, so the result would
// depend on which recovery rows are read; root.zig:268-335 reads all of them)
namespace {
// decode_betas solves a small GF(2^16) system per code: memoised per (k, m), since every
// reconstruct call asks
bool has_decode_betas(uint64_t k, uint64_t m) {
  static std::mutex mu;
  static std::unordered_map<uint64_t, bool> memo;
  const uint64_t key = k << 32 | m;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = memo.find(key);
    if (it != memo.end()) return it->second;
  }
  std::vector<uint16_t> beta;
  const bool ok = fftnet::decode_betas(static_cast<uint32_t>(k), static_cast<uint32_t>(m), beta);
  std::lock_guard<std::mutex> lk(mu);
  memo[key] = ok;
  return ok;
}
}  // namespace

bool fdec_supports(uint64_t k, uint64_t m, uint64_t sb, uint32_t flags) {
  const uint64_t C = ceil_pow2(m);
  const bool d2_drops = (flags & RS_FLAG_QUIRK_D2) && k > C && k % C == 0;
  return fdec_mode() != 0 && !(flags & RS_FLAG_QUIRK_D1) && !d2_drops && fft_enabled() &&
         fftnet::supports(k, m, sb, true) && fftnet::pieces(sb) == 1 && sb % fftnet::kUnitBytes == 0 &&
         has_decode_betas(k, m);
}

const jit::Kernel *wps_solve_kernel(WpsSlot &ws) {
  std::lock_guard<std::mutex> lk(ws.mu);
  if (ws.solve_failed) return nullptr;
  std::string err;
  const jit::Kernel *sk = psyn::get_solve(cantor_basis(), err);
  if (!sk) {
    ws.solve_failed = true;
    warn_once_per_reason("[rs_amd] per-stripe solve kernel unavailable, using table kernels: ", err);
  }
  return sk;
}

}  // namespace host
}  // namespace rs

namespace {
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
  alloc_point();
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
  bool pending = false;
  const jit::Kernel *k = psyn::get(p.spec, err, pending);
  if (!k && !pending) {
    p.failed = true;
    warn_once_per_reason("[rs_amd] per-stripe syndrome network unavailable, using table kernels: ", err);
  }
  return k;
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
         (mode.empty() || mode == "auto" || mode == "psyn") && fft_enabled() && fftnet::supports(k, m, sb, true) &&
         fftnet::pieces(sb) == 1 && sb % jit::kUnitBytes == 0 &&
         m <= 64;  // max_e up to m: output groups of 8 (rs_psyn.hpp launch_solve)
}

// the fused FFT reconstruct with per-stripe decode blocks (any whole 2 KiB units). Its
// decode tail costs about the same for any loss count (an IFFT plus one FFT per data block
// with a loss), the generic solve grows with max_e^2. Per-stripe random patterns, 256 KiB
// x 256 (profiles/r03/fdec/patterns_*.jsonl), fused vs solve: RS(200,55) max_e 20 / 30 /
// 40 / 55: 6.6 / 6.9 / 7.3 / 7.7 vs 4.8 / 6.6 / 9.0 / 14.0 ms; RS(64,64) max_e 20 / 40:
// 3.0 / 3.6 vs 2.2 / 4.0 ms; RS(100,20) max_e 20: 3.2 vs 3.3 ms. So auto takes it for
// max_e >= 0.6 m (and where the solve has no 4 KiB units to run on); RS_AMD_FDEC=1 always.
bool fdec_patterns_enabled(uint64_t k, uint64_t m, uint64_t sb, uint32_t flags, uint32_t max_e) {
  const char *pm = std::getenv("RS_AMD_PATTERNS");
  const std::string mode = pm ? pm : "";
  if (!(mode.empty() || mode == "auto" || mode == "psyn") || m > 64 || !fdec_supports(k, m, sb, flags)) return false;
  return fdec_mode() == 1 || 5ull * max_e >= 3ull * m || sb % jit::kUnitBytes != 0;
}

bool psyn_enabled(uint64_t k, uint64_t m, uint64_t sb, uint32_t flags) {
  const char *pm = std::getenv("RS_AMD_PATTERNS");
  const std::string mode = pm ? pm : "";
  return !(flags & RS_FLAG_QUIRK_D1) && !d2_drops_chunk(k, m, flags) &&
         (mode.empty() || mode == "auto" || mode == "psyn") && jit::enabled() && psyn::supports(k, m, sb);
}

}  // namespace

void rs::host::release_patterns() {
  std::lock_guard<std::mutex> lk(g_plan_mu);
  g_dev_tables.clear();
  g_wps.clear();
  g_psyn_plans.clear();
}

extern "C" {

const char *rs_patterns_kernel_name(uint64_t k, uint64_t m, size_t sb, uint32_t max_e, uint32_t flags) {
  thread_local std::string name;
  if (is_low_rate(k, m)) {
    name = "pattern_fft_low";
  } else if (psyn_enabled(k, m, sb, flags)) {
    name = "psyn_k" + std::to_string(k) + "_m" + std::to_string(m);
  } else if (fdec_patterns_enabled(k, m, sb, flags, max_e)) {
    name = "fft_decode";
  } else if (wps_enabled(k, m, sb, flags, max_e)) {
    name = "fft_syndromes+psyn_solve";
  } else {
    const char *pm = std::getenv("RS_AMD_PATTERNS");
    const uint64_t W = ceil_pow2(ceil_pow2(m) + k);
    const bool matrix =
        !literal_decode(k, m, flags) && W <= 32 && max_e <= kMatrixMaxOut && !(pm && std::string(pm) == "fft");
    name = matrix ? "pattern_matrix" : "pattern_fft";
  }
  return name.c_str();
}

int rs_reconstruct_batch_dev_patterns(uint64_t k, uint64_t m, size_t sb, uint64_t n_stripes, const uint8_t *d_present,
                                      uint64_t present_stride, uint32_t max_e, const void *d_original,
                                      uint64_t orig_stride, const void *d_recovery, uint64_t rec_stride,
                                      void *d_restored, uint64_t out_stride, int32_t *d_status, uint32_t flags,
                                      rs_stream_t stream) {
  TraceScope ts;
  return guarded([&]() -> int {
    int st = check_codec(k, m, sb);
    if (st) return st;
    const bool low = is_low_rate(k, m);  // §8 f4: the low-rate layout on the FFT kernels only
    if (n_stripes == 0 || max_e == 0) return RS_OK;
    if (!d_present || !d_original || !d_recovery || !d_restored) return fail(RS_ERR_INVALID_ARGUMENT, "NULL pointer");
    if (present_stride == 0) present_stride = k + m;
    if (orig_stride == 0) orig_stride = k * sb;
    if (rec_stride == 0) rec_stride = m * sb;
    if (out_stride == 0) out_stride = static_cast<uint64_t>(max_e) * sb;
    if (sb % 64) {  // shard tails (root.zig:338-348 layout): padded copies, in slices
      int dev;
      if ((st = current_device(&dev))) return st;
      hipStream_t s = static_cast<hipStream_t>(stream);
      const uint64_t psb = (sb + 63) / 64 * 64, rows = k + m + max_e;
      const uint64_t cap = std::max<uint64_t>(1, std::min<uint64_t>(n_stripes, kTailSliceBytes / (rows * psb)));
      void *buf = nullptr;
      HIP_TRY(dev_malloc_async(&buf, cap * rows * psb, s));
      uint8_t *po = static_cast<uint8_t *>(buf), *pr = po + cap * k * psb, *pout = pr + cap * m * psb;
      const uint8_t *O = static_cast<const uint8_t *>(d_original), *Rc = static_cast<const uint8_t *>(d_recovery);
      uint8_t *Out = static_cast<uint8_t *>(d_restored);
      for (uint64_t s0 = 0; st == RS_OK && s0 < n_stripes; s0 += cap) {
        const uint64_t cnt = std::min(cap, n_stripes - s0);
        // every slot is padded (which are present varies per stripe; the kernels read only
        // those), and the restored rows too, so the slots a stripe does not restore come
        // back unchanged
        for (uint64_t i = 0; st == RS_OK && i < k; i++)
          st = pad_shards(O + s0 * orig_stride + i * sb, orig_stride, sb, po + i * psb, k * psb, psb, cnt, s);
        for (uint64_t i = 0; st == RS_OK && i < m; i++)
          st = pad_shards(Rc + s0 * rec_stride + i * sb, rec_stride, sb, pr + i * psb, m * psb, psb, cnt, s);
        for (uint64_t j = 0; st == RS_OK && j < max_e; j++)
          st = pad_shards(Out + s0 * out_stride + j * sb, out_stride, sb, pout + j * psb, max_e * psb, psb, cnt, s);
        if (st == RS_OK)
          st = rs_reconstruct_batch_dev_patterns(k, m, psb, cnt, d_present + s0 * present_stride, present_stride, max_e,
                                                 po, 0, pr, 0, pout, 0, d_status ? d_status + s0 : nullptr, flags,
                                                 stream);
        for (uint64_t j = 0; st == RS_OK && j < max_e; j++)
          st = unpad_shards(pout + j * psb, max_e * psb, sb, Out + s0 * out_stride + j * sb, out_stride, cnt, s);
      }
      (void)hipFreeAsync(buf, s);
      return st;
    }
    const int max_nv = align_nv({reinterpret_cast<uint64_t>(d_original), reinterpret_cast<uint64_t>(d_recovery),
                                 reinterpret_cast<uint64_t>(d_restored), orig_stride, rec_stride, out_stride});
    if (!max_nv) return fail(RS_ERR_INVALID_ARGUMENT, "device pointers/strides must be 4-byte aligned");
    int dev;
    if ((st = current_device(&dev))) return st;
    const uint64_t C = low ? ceil_pow2(k) : ceil_pow2(m), W = ceil_pow2(low ? C + m : C + k);
    const uint16_t *dexp, *dlog, *dlw;
    if ((st = device_tables(dev, &dexp, &dlog, &dlw))) return st;
    if (low) flags &= ~(RS_FLAG_QUIRK_D1 | RS_FLAG_QUIRK_D2);  // no literal low-rate behaviour (rs_lowrate.cpp)
    // syndrome network (rs_psyn.hpp): the code's fixed k -> m network plus a per-stripe
    // e x e solve; corrected multiply, k <= 64, m <= 4, whole 4 KiB units
    if (!low && max_nv == 4 && psyn_enabled(k, m, sb, flags)) {
      std::shared_ptr<PsynPlan> pp;
      if ((st = psyn_plan(dev, k, m, flags, pp))) return st;
      if (const jit::Kernel *pk = psyn_kernel(*pp)) {
        hipStream_t s = static_cast<hipStream_t>(stream);
        const uint32_t mo = psyn::max_out(static_cast<uint32_t>(k), static_cast<uint32_t>(m));
        const uint32_t pdw = psyn::plan_dwords(static_cast<uint32_t>(k), static_cast<uint32_t>(m));
        void *blk = nullptr;
        HIP_TRY(dev_malloc_async(&blk, n_stripes * pdw * sizeof(uint32_t), s));
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
    // wide codes: the fused FFT reconstruct with per-stripe decode blocks built on the GPU
    // (trimmed rows R, erasure locator, masks)
    if (!low && max_nv == 4 && fdec_patterns_enabled(k, m, sb, flags, max_e)) {
      std::shared_ptr<WpsSlot> ws;
      wps_slot(dev, k, m, flags, ws);
      const fftnet::Spec *dfs = nullptr;
      // blocked unit walk: a workgroup takes one stripe's units in a row, so the stripe's
      // decode block stays in the scalar cache (RS(200,55) max_e 55: 10.0 -> 7.7 ms,
      // RS(64,64) max_e 40: 4.75 -> 3.59 ms; for a batch-wide block it changes nothing,
      // 6.91 vs 6.91 ms; profiles/r03/fdec/)
      if (const jit::Kernel *fk = fft_kernel(*ws->decb, sb, &dfs)) {
        hipStream_t s = static_cast<hipStream_t>(stream);
        const uint32_t words = fftnet::decode_block_words(*dfs), dwm = fftnet::dyn_mask_words(*dfs),
                       mko = fftnet::decode_mask_offset(*dfs);
        FdecConsts cst{};
        std::vector<uint16_t> beta;
        fftnet::decode_betas(static_cast<uint32_t>(k), static_cast<uint32_t>(m), beta);
        for (size_t i = 0; i < beta.size() && i < 32; i++) cst.beta[i] = beta[i];
        fftnet::uv_basis(cst.p);
        // decode blocks in slices of <= 1 GiB
        const uint64_t per_bytes = static_cast<uint64_t>(words) * 4 + (k + m) + W * 2;
        const uint64_t per = std::max<uint64_t>(1, std::min<uint64_t>(n_stripes, (1ull << 30) / per_bytes));
        void *tmp = nullptr;
        HIP_TRY(dev_malloc_async(&tmp, per * per_bytes + 256, s));
        uint32_t *blk = static_cast<uint32_t *>(tmp);
        uint16_t *logs = reinterpret_cast<uint16_t *>(blk + per * words);
        uint8_t *trimmed = reinterpret_cast<uint8_t *>(logs + per * W);
        hipError_t e = hipSuccess;
        for (uint64_t s0 = 0; e == hipSuccess && s0 < n_stripes; s0 += per) {
          const uint64_t cnt = std::min(per, n_stripes - s0);
          e = launch_fdec_plan(d_present + s0 * present_stride, present_stride, static_cast<uint32_t>(k),
                               static_cast<uint32_t>(m), static_cast<uint32_t>(C), static_cast<uint32_t>(W), cnt, max_e,
                               dexp, dlog, dlw, trimmed, logs, blk, dwm, mko, words, cst,
                               d_status ? d_status + s0 : nullptr, s);
          if (e == hipSuccess)
            e = fftnet::launch(*fk, *dfs, static_cast<const uint8_t *>(d_original) + s0 * orig_stride, orig_stride,
                               static_cast<const uint8_t *>(d_recovery) + s0 * rec_stride, rec_stride,
                               static_cast<uint8_t *>(d_restored) + s0 * out_stride, out_stride, sb, cnt, s, blk, words);
        }
        (void)hipFreeAsync(tmp, s);
        if (e != hipSuccess) return hip_fail(e, "per-stripe fused FFT reconstruct");
        return RS_OK;
      }
      if (fdec_mode() == 1) return fail(RS_ERR_DEVICE, "RS_AMD_FDEC=1: fused FFT reconstruct kernel unavailable");
    }
    // wide codes: syndromes on the FFT kernel (per-stripe masks), then the e x e solve
    if (!low && max_nv == 4 && wps_enabled(k, m, sb, flags, max_e)) {
      std::shared_ptr<PsynPlan> pp;  // G and the Cantor basis
      if ((st = psyn_plan(dev, k, m, flags, pp))) return st;
      std::shared_ptr<WpsSlot> ws;
      wps_slot(dev, k, m, flags, ws);
      const fftnet::Spec *fs = nullptr;
      const jit::Kernel *fk = fft_kernel(*ws->fft, sb, &fs);
      const jit::Kernel *sk = wps_solve_kernel(*ws);
      if (fk && sk) {
        hipStream_t s = static_cast<hipStream_t>(stream);
        // coefficients for min(max_e, m) outputs per syndrome, in groups of 8
        const uint32_t cs = wps_coef_stride(static_cast<uint32_t>(std::min<uint64_t>(max_e, m)));
        const uint32_t dmw = fftnet::dyn_mask_words(*fs), pw = dmw + 2 + 64 + 64 * cs;
        const uint64_t per = std::max<uint64_t>(1, std::min<uint64_t>(n_stripes, kScratchCap / (m * sb)));
        void *blk = nullptr, *scratch = nullptr;
        HIP_TRY(dev_malloc_async(&blk, n_stripes * pw * sizeof(uint32_t), s));
        hipError_t e = dev_malloc_async(&scratch, per * m * sb, s);
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
    const bool use_matrix = !low && !literal_decode(k, m, flags) && W <= 32 && max_e <= kMatrixMaxOut &&
                            !(pm && std::string(pm) == "fft");
    // per-stripe plan: logs u16 | pre RsTab | post RsTab | src i32 | dst i32 (W entries each)
    //                  [| trimmed present rows, matrix path]
    const uint64_t per = W * (2 + 2 * sizeof(RsTab) + 8);
    void *tmp = nullptr;
    HIP_TRY(dev_malloc_async(&tmp, n_stripes * per + (use_matrix ? n_stripes * (k + m) : 0) + 256, s));
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
                                       flags & RS_FLAG_QUIRK_D1, low, dexp, dlog, dlw, logs, pre, post, src, dst,
                                       d_status, s);
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
      e = dev_malloc_async(&mt, tab_bytes + img_bytes + nk * 4 + n_stripes * 4 + 256, s);
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
    const KernelChoice kc = low ? choose_decode_w(W, sb, max_nv) : choose_decode(k, m, sb, max_nv);
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
    a.trunc = static_cast<uint32_t>(low ? C + m : C + k);
    a.trunc_fft = low ? static_cast<uint32_t>(k) : 0;  // as rs_lowrate.cpp low_reconstruct
    a.pattern_stride = W;
    a.contig = kc.variant != Variant::kGeneric && contig_ok(sb, kc.nv);
    if (kc.variant != Variant::kGeneric) {
      a.n_stripes = n_stripes;
      e = launch_decode(kc, a, s);
    } else {
      // launch_decode_generic: the transform plus the FFT's kept rows, per stripe
      const uint64_t rows = decode_generic_rows(W, a.trunc, a.trunc_fft);
      const uint64_t cap = slice_stripes(n_stripes, rows * sb);
      void *scratch = nullptr;
      e = dev_malloc_async(&scratch, cap * rows * sb, s);
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

}  // extern "C"
