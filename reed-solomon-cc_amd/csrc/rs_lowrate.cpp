// rs_lowrate.cpp — the low-rate codec (§8 f4): pow2(k) < pow2(m), or equal with k > m.
//
// The reference panics here (root.zig:119-121, 226-228) and vendors no low-rate code, so
// this is the low-rate codec of the algorithm it ports (reed-solomon-simd, named in
// benchmarks.zig:1-2): PARITY UNPINNED, no reference output exists. Quirk flags are
// ignored (D1 / D2 are defects of the reference's high-rate path; there is no literal
// low-rate behaviour to reproduce): the corrected multiply always.
//
//  * encode (rs_gf.hpp scalar_encode_low): originals at positions [0, k) of one chunk
//    C = ceilPow2(k), coefficients = IFFT(C, trunc k, skew 0), recovery chunk j =
//    FFT(coefficients, trunc min(C, m - jC), skew (j + 1) C). FFT-form kernels
//    (rs_kernels.hip k_encode_low_reg for C <= 32, k_encode_low_generic otherwise).
//  * reconstruct (rs_gf.hpp scalar_reconstruct_low): the erasure-locator decode of
//    root.zig:268-335 in the low-rate position layout (recovery at [C, C + m), [C + m, W)
//    erased), on the decode kernels with the FFT truncated to k (k_decode_reg for
//    W <= 32, launch_decode_generic otherwise) — no host solve, any (k, m) useHighRate accepts.
//  * small codes: a bit-sliced network of the encode map (<= 64 outputs) and of each
//    erasure pattern's reconstruct map (<= 64 restored, by GF(2) linear algebra on the
//    host), HBM-bound; the FFT-form kernels run until such a network is compiled.
#include "rs_host.hpp"

namespace rs {
namespace host {

namespace {

// single-pass maps only (every output of the map in one network kernel)
bool map_net_ok(uint64_t n_in, uint64_t n_out, uint64_t sb) {
  return jit::enabled() && n_out > 0 && n_out <= jit::kMaxOut &&
         jit::supports_async(static_cast<uint32_t>(n_in), static_cast<uint32_t>(n_out), sb);
}

struct LowEncodePlan {
  std::shared_ptr<DevBuf> tabs;  // IFFT(C, skew 0), then FFT(C, skew (j+1)C) per recovery chunk
  uint32_t C = 0, n_chunks = 0, tabs_per_chunk = 0;
  std::shared_ptr<NetSlot> net;  // the encode map's network (small codes)
};

struct LowDecodePlan {
  std::shared_ptr<DevBuf> tw;    // IFFT + FFT tables of size W (shared per W)
  std::shared_ptr<DevBuf> buf;   // pre[W] | post[W] RsTab, src[W] | dst[W] int32
  size_t off_fft = 0;
  uint32_t W = 0, trunc = 0, e = 0;
  std::shared_ptr<NetSlot> net;  // the pattern's reconstruct map (small codes)
  // the block form (launch_low_blocks), when block_ok: one device blob at the off_* offsets
  bool block = false;
  uint32_t C = 0, n_blocks = 0, mprime = 0;
  std::vector<uint8_t> u, used;  // per block: u (host scalar form), some recovery row read
  std::shared_ptr<DevBuf> bbuf;
  size_t off_i = 0, off_f = 0, off_gamma = 0, off_gamma1 = 0, off_syn = 0, off_post = 0, off_sidx = 0, off_dst = 0,
         off_skip = 0;
};

PlanCache<LowEncodePlan> g_low_enc;
PlanCache<LowDecodePlan> g_low_dec;  // a W = 65536 plan holds 13 MB of HBM: plans are LRU-capped

}  // namespace

void release_lowrate() {
  std::lock_guard<std::mutex> lk(g_plan_mu);
  g_low_enc.clear();
  g_low_dec.clear();
}

void encode_low_map(uint64_t k, uint64_t m, uint32_t flags, jit::NetSpec &ns) {
  (void)flags;  // corrected multiply (quirks have no low-rate meaning)
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
      scalar_encode_low(in.data(), k, m, false, out.data());
      for (uint64_t j = 0; j < m; j++) ns.images[(t * m + j) * 16 + b] = out[j];
    }
    in[t] = 0;
  }
}

namespace {
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

}  // namespace

int low_decode_map(uint64_t k, uint64_t m, uint32_t flags, const uint8_t *present, jit::NetSpec &ns) {
  jit::NetSpec G;
  encode_low_map(k, m, flags, G);
  return linear_decode_map(k, m, G, present, "reconstruct_low", ns);
}

namespace {

int get_low_encode_plan(int dev, uint64_t k, uint64_t m, uint64_t sb, std::shared_ptr<LowEncodePlan> &out) {
  const bool net = map_net_ok(k, m, sb);
  const std::string key = std::to_string(dev) + "/" + std::to_string(k) + "/" + std::to_string(m) + "/" +
                          std::to_string(net) + "/" + std::to_string(jit::max_blocks());
  {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    if ((out = g_low_enc.find(key))) return RS_OK;
  }
  alloc_point();
  auto p = std::make_shared<LowEncodePlan>();
  const uint64_t C = ceil_pow2(k);
  p->C = static_cast<uint32_t>(C);
  p->n_chunks = static_cast<uint32_t>((m + C - 1) / C);
  p->tabs_per_chunk = static_cast<uint32_t>(fft_tab_count(C));
  std::vector<RsTab> tabs;
  push_ifft_tabs(tabs, C, 0, false);
  for (uint64_t j = 0; j < p->n_chunks; j++) push_fft_tabs(tabs, C, (j + 1) * C, false);
  if (tabs.empty()) tabs.push_back(make_twiddle(kModulus, false));  // C = 1: no butterflies
  if (int st = upload(tabs.data(), tabs.size() * sizeof(RsTab), dev, p->tabs)) return st;
  if (net) {
    p->net = std::make_shared<NetSlot>();
    p->net->async = !jit::supports(static_cast<uint32_t>(k), static_cast<uint32_t>(m), sb);
    encode_low_map(k, m, 0, p->net->spec);
  }
  std::lock_guard<std::mutex> lk(g_plan_mu);
  out = g_low_enc.insert(key, p);
  return RS_OK;
}

// the block form: C-point transforms only (C >= 128: launch_low_blocks' phase shapes), any
// number of blocks up to kLowBlockMaxBlocks; RS_AMD_LOW_BLOCK=0 keeps the W-point decode
bool block_ok(uint64_t k, uint64_t m, uint64_t sb) {
  const char *ev = std::getenv("RS_AMD_LOW_BLOCK");
  if (ev && std::strcmp(ev, "0") == 0) return false;
  const uint64_t C = ceil_pow2(k), W = ceil_pow2(C + m);
  return C >= 128 && W / C <= kLowBlockMaxBlocks && sb % 64 == 0;
}

// the block form serves a pattern when its shapes fit (block_ok) and the rows read are
// trimmed to the first e present (RS_AMD_LOW_TRIM); shared by get_low_decode_plan and the
// kernel-name prediction. Its work grows with the blocks holding a row read only
// (launch_low_blocks skips the others), at most ceil(m / C) < W / C of them, so it stays
// below the W-point decode's transforms for every pattern.
bool block_form(uint64_t k, uint64_t m, uint64_t sb, uint64_t e) {
  const char *te = std::getenv("RS_AMD_LOW_TRIM");
  return !(te && std::strcmp(te, "0") == 0) && e > 0 && block_ok(k, m, sb);
}

uint16_t log_of(uint16_t x) { return tables().log[x]; }

// the device blob of the block form (layout: LowDecodePlan::off_*)
int build_block_plan(int dev, uint64_t k, uint64_t m, const uint8_t *received, const uint16_t *er, LowDecodePlan &p) {
  const uint64_t C = ceil_pow2(k);
  uint64_t mp = 0;  // the last recovery row used + 1
  for (uint64_t r = 0; r < m; r++)
    if (received[C + r]) mp = r + 1;
  if (mp == 0) return RS_OK;  // nothing erased: no block form needed
  const uint64_t nbk = (mp + C - 1) / C;
  std::vector<uint16_t> alpha, beta;
  low_block_coefs(k, m, alpha, beta);
  std::vector<RsTab> tabs;
  push_ifft_tabs(tabs, C, 0, false);  // the low-rate encode's tables (launch_encode_low_phases)
  for (uint64_t j = 0; j < nbk; j++) push_fft_tabs(tabs, C, (j + 1) * C, false);
  const size_t n_e = tabs.size();
  for (uint64_t j = 0; j < nbk; j++) push_ifft_tabs(tabs, C, (j + 1) * C, false);
  const size_t n_i = tabs.size() - n_e;
  push_fft_tabs(tabs, C, 0, false);
  const size_t n_f = tabs.size() - n_e - n_i;
  uint16_t zimg[16] = {};
  const RsTab zero = make_tab_from_images(zimg);
  p.u.assign(nbk, 0);
  p.used.assign(nbk, 0);
  for (uint64_t r = 0; r < mp; r++)
    if (received[C + r]) p.used[r / C] = 1;
  std::vector<uint16_t> sig(nbk, 0);
  for (uint64_t j = 0; j < nbk; j++) {  // gamma: sigma_K = alpha_K (u = 1) or beta_K (u = 0)
    const uint16_t al = alpha[j + 1], be = beta[j + 1];
    if (al) {
      p.u[j] = 1;
      sig[j] = al;
      tabs.push_back(be ? make_tab(static_cast<uint16_t>((log_of(be) + kModulus - log_of(al)) % kModulus), false) : zero);
    } else {
      sig[j] = be;  // both zero: the block adds nothing (its syndromes are scaled to zero)
      tabs.push_back(make_tab(0, false));
    }
  }
  for (uint64_t j = 0; j < nbk; j++) {  // 1 + gamma (k_ephase DLO: W = ((1 + gamma) I + D_lo) U)
    const uint16_t al = alpha[j + 1], be = beta[j + 1];
    const uint16_t gv = al && be ? tables().exp[(log_of(be) + kModulus - log_of(al)) % kModulus] : 0;
    const uint16_t g1 = static_cast<uint16_t>(1u ^ gv);
    tabs.push_back(p.u[j] && g1 ? make_tab(log_of(g1), false) : zero);
  }
  std::vector<int32_t> sidx(nbk * C, -1), dst(C, -1);
  const size_t at_syn = tabs.size();
  tabs.resize(at_syn + nbk * C + C, zero);
  for (uint64_t r = 0; r < mp; r++)
    if (received[C + r]) {
      sidx[r] = 1;
      const uint16_t sg = sig[r / C];
      tabs[at_syn + r] = sg ? make_tab(static_cast<uint16_t>((er[C + r] + log_of(sg)) % kModulus), false) : zero;
    }
  int32_t ne = 0;
  std::vector<uint32_t> skip((k + 31) / 32, 0);
  for (uint64_t g = 0; g < k; g++)
    if (!received[g]) {
      dst[g] = ne++;
      tabs[at_syn + nbk * C + g] = make_tab(static_cast<uint16_t>(kModulus - er[g]), false);
      skip[g / 32] |= 1u << (g % 32);
    }
  p.off_i = n_e * sizeof(RsTab);
  p.off_f = (n_e + n_i) * sizeof(RsTab);
  p.off_gamma = (n_e + n_i + n_f) * sizeof(RsTab);
  p.off_gamma1 = p.off_gamma + nbk * sizeof(RsTab);
  p.off_syn = at_syn * sizeof(RsTab);
  p.off_post = (at_syn + nbk * C) * sizeof(RsTab);
  p.off_sidx = tabs.size() * sizeof(RsTab);
  p.off_dst = p.off_sidx + sidx.size() * sizeof(int32_t);
  p.off_skip = p.off_dst + dst.size() * sizeof(int32_t);
  std::vector<uint8_t> blob(p.off_skip + skip.size() * sizeof(uint32_t));
  std::memcpy(blob.data(), tabs.data(), tabs.size() * sizeof(RsTab));
  std::memcpy(blob.data() + p.off_sidx, sidx.data(), sidx.size() * sizeof(int32_t));
  std::memcpy(blob.data() + p.off_dst, dst.data(), dst.size() * sizeof(int32_t));
  std::memcpy(blob.data() + p.off_skip, skip.data(), skip.size() * sizeof(uint32_t));
  if (int st = upload(blob.data(), blob.size(), dev, p.bbuf)) return st;
  p.block = true;
  p.C = static_cast<uint32_t>(C);
  p.n_blocks = static_cast<uint32_t>(nbk);
  p.mprime = static_cast<uint32_t>(mp);
  return RS_OK;
}

int get_low_decode_plan(int dev, uint64_t k, uint64_t m, uint64_t sb, const uint8_t *present,
                        std::shared_ptr<LowDecodePlan> &out) {
  uint64_t e = 0;
  for (uint64_t i = 0; i < k; i++) e += present[i] ? 0 : 1;
  const bool net = map_net_ok(k, e, sb);
  const char *te = std::getenv("RS_AMD_LOW_TRIM");
  const bool trim = !(te && std::strcmp(te, "0") == 0);
  const bool blk = block_form(k, m, sb, e);
  std::string key = std::to_string(dev) + "/" + std::to_string(k) + "/" + std::to_string(m) + "/" +
                    std::to_string(net) + "/" + std::to_string(jit::max_blocks()) + "/" + (trim ? "t/" : "a/") +
                    (blk ? "b/" : "w/");
  key.reserve(key.size() + k + m);
  for (uint64_t i = 0; i < k + m; i++) key.push_back(present[i] ? '1' : '0');
  {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    if ((out = g_low_dec.find(key))) return RS_OK;
  }
  alloc_point();
  auto p = std::make_shared<LowDecodePlan>();
  const uint64_t C = ceil_pow2(k), end = C + m, W = ceil_pow2(end);
  p->W = static_cast<uint32_t>(W);
  // position layout of scalar_reconstruct_low: originals [0, k), recovery [C, C + m). Only
  // the first e present recovery rows are read (round 5): with the k - e present originals and
  // the known zeros [k, C) that is exactly C known positions, the dimension of the code, and
  // the restored originals are the same; the other present rows join the erasures. Nothing is
  // received past the last row read, so the IFFT is truncated there (its groups past it are
  // all zero, Generic.zig:80-147), and its gather reads k rows instead of every present one.
  // (RS_AMD_LOW_TRIM=0: every present row, the IFFT truncated at C + m, as before round 5)
  std::vector<uint8_t> received(W, 0);
  for (uint64_t i = 0; i < k; i++) received[i] = present[i] ? 1 : 0;
  uint64_t last = k, nr = 0;
  for (uint64_t r = 0; r < m && (nr < e || !trim); r++)
    if (present[k + r]) received[C + r] = 1, nr++, last = C + r + 1;
  p->trunc = static_cast<uint32_t>(trim ? last : end);
  std::vector<uint16_t> er(kOrder);
  erasure_logs_low(received.data(), k, m, er.data());
  if (blk) {  // the block form needs none of the W-point tables
    if (int st = build_block_plan(dev, k, m, received.data(), er.data(), *p)) return st;
  }
  if (!p->block) {
    if (int st = twiddle_plan(dev, W, 0, p->tw, p->off_fft)) return st;
  }
  std::vector<RsTab> tabs(2 * W);  // pre, post
  std::vector<int32_t> idx(2 * W, -1);  // src, dst
  uint32_t ne = 0;
  for (uint64_t q = 0; q < W; q++) {
    if (q < k && received[q]) {
      idx[q] = static_cast<int32_t>(q);
      tabs[q] = make_tab(er[q], false);
    } else if (q >= C && q < end && received[q]) {
      idx[q] = kSrcRecovery | static_cast<int32_t>(q - C);
      tabs[q] = make_tab(er[q], false);
    }
    if (q < k && !received[q]) {
      idx[W + q] = static_cast<int32_t>(ne++);
      tabs[W + q] = make_tab(static_cast<uint16_t>(kModulus - er[q]), false);
    }
  }
  p->e = ne;
  if (!p->block) {
    std::vector<uint8_t> blob(tabs.size() * sizeof(RsTab) + idx.size() * sizeof(int32_t));
    std::memcpy(blob.data(), tabs.data(), tabs.size() * sizeof(RsTab));
    std::memcpy(blob.data() + tabs.size() * sizeof(RsTab), idx.data(), idx.size() * sizeof(int32_t));
    if (int st = upload(blob.data(), blob.size(), dev, p->buf)) return st;
  }
  if (net) {
    p->net = std::make_shared<NetSlot>();
    p->net->async = !jit::supports(static_cast<uint32_t>(k), static_cast<uint32_t>(e), sb);
    if (int st = low_decode_map(k, m, 0, present, p->net->spec)) return st;
  }
  std::lock_guard<std::mutex> lk(g_plan_mu);
  out = g_low_dec.insert(key, p);
  return RS_OK;
}

// generic kernels walk a scratch of `per_stripe` positions x sb per stripe, in slices
template <class F>
int in_scratch_slices(uint64_t n, uint64_t per_stripe_bytes, hipStream_t s, F &&launch) {
  const uint64_t per = slice_stripes(n, per_stripe_bytes);
  void *scratch = nullptr;
  HIP_TRY(dev_malloc_async(&scratch, per * per_stripe_bytes, s));
  hipError_t e = hipSuccess;
  for (uint64_t s0 = 0; e == hipSuccess && s0 < n; s0 += per)
    e = launch(s0, std::min(per, n - s0), static_cast<uint8_t *>(scratch));
  (void)hipFreeAsync(scratch, s);
  return e == hipSuccess ? RS_OK : hip_fail(e, "low-rate generic kernel");
}

}  // namespace

int low_encode(int dev, uint64_t k, uint64_t m, uint64_t sb, uint64_t n, const uint8_t *orig, uint64_t ostride,
               uint8_t *rec, uint64_t rstride, uint32_t flags, int max_nv, hipStream_t s) {
  (void)flags;
  std::shared_ptr<LowEncodePlan> p;
  if (int st = get_low_encode_plan(dev, k, m, sb, p)) return st;
  if (p->net && max_nv == 4)
    if (const jit::Kernel *nk = net_kernel(*p->net, sb)) {
      HIP_TRY(jit::launch(*nk, orig, ostride, nullptr, 0, rec, rstride, sb, n, s));
      return RS_OK;
    }
  const KernelChoice kc = choose_encode_low(p->C, sb, max_nv);
  EncodeArgs a{};
  a.data = orig;
  a.data_stripe_stride = ostride;
  a.parity = rec;
  a.parity_stripe_stride = rstride;
  a.shard_bytes = sb;
  a.tabs = static_cast<const RsTab *>(p->tabs->p);
  a.chunk = p->C;
  a.n_chunks = p->n_chunks;
  a.tabs_per_chunk = p->tabs_per_chunk;
  a.k = static_cast<uint32_t>(k);
  a.m = static_cast<uint32_t>(m);
  a.contig = kc.variant != Variant::kGeneric && contig_ok(sb, kc.nv);
  if (kc.variant != Variant::kGeneric) {
    a.n_stripes = n;
    HIP_TRY(launch_encode_low(kc, a, s));
    return RS_OK;
  }
  // coefficients + one intermediate region per recovery chunk (the chunks' FFTs run in
  // parallel), in groups of G chunks so that a stripe's (1 + G) regions fit the scratch cap
  // (G = 1 at least: two regions per stripe)
  const uint64_t region = static_cast<uint64_t>(p->C) * sb;
  const uint64_t fit = scratch_cap() / region;  // regions of one stripe that fit the cap
  const uint64_t G = std::max<uint64_t>(1, std::min<uint64_t>(p->n_chunks, fit > 1 ? fit - 1 : 1));
  a.regions = static_cast<uint32_t>(1 + G);
  return in_scratch_slices(n, (1 + G) * region, s, [&](uint64_t s0, uint64_t cnt, uint8_t *scratch) {
    EncodeArgs b = a;
    b.data += s0 * ostride;
    b.parity += s0 * rstride;
    b.n_stripes = cnt;
    b.scratch = scratch;
    return launch_encode_low(kc, b, s);
  });
}

int low_reconstruct(int dev, uint64_t k, uint64_t m, uint64_t sb, uint64_t n, const uint8_t *present,
                    const uint8_t *orig, uint64_t ostride, const uint8_t *rec, uint64_t rstride, uint8_t *out,
                    uint64_t outstride, uint32_t flags, int max_nv, hipStream_t s) {
  (void)flags;
  std::shared_ptr<LowDecodePlan> p;
  if (int st = get_low_decode_plan(dev, k, m, sb, present, p)) return st;
  if (!orig) orig = rec;  // never dereferenced for absent shards
  if (!rec) rec = orig;
  if (p->net && max_nv == 4)
    if (const jit::Kernel *nk = net_kernel(*p->net, sb)) {
      HIP_TRY(jit::launch(*nk, orig, ostride, rec, rstride, out, outstride, sb, n, s));
      return RS_OK;
    }
  if (p->block) {
    const uint8_t *base = static_cast<const uint8_t *>(p->bbuf->p);
    LowBlockArgs L{};
    EncodeArgs &a = L.enc;
    a.data = orig;
    a.data_stripe_stride = ostride;
    a.shard_bytes = sb;
    a.tabs = reinterpret_cast<const RsTab *>(base);
    a.chunk = p->C;
    a.n_chunks = p->n_blocks;
    a.tabs_per_chunk = static_cast<uint32_t>(fft_tab_count(p->C));
    a.k = static_cast<uint32_t>(k);
    a.m = p->mprime;
    a.skip = reinterpret_cast<const uint32_t *>(base + p->off_skip);
    DecodeArgs &d = L.dec;
    d.out = out;
    d.out_stripe_stride = outstride;
    d.shard_bytes = sb;
    d.tab_fft = reinterpret_cast<const RsTab *>(base + p->off_f);
    d.tab_post = reinterpret_cast<const RsTab *>(base + p->off_post);
    d.pos_dst = reinterpret_cast<const int32_t *>(base + p->off_dst);
    d.contig = contig_ok(sb, 1);
    L.rec = rec;
    L.rec_stripe_stride = rstride;
    L.syn_idx = reinterpret_cast<const int32_t *>(base + p->off_sidx);
    L.syn_tab = reinterpret_cast<const RsTab *>(base + p->off_syn);
    L.tabs_i = reinterpret_cast<const RsTab *>(base + p->off_i);
    L.gamma = reinterpret_cast<const RsTab *>(base + p->off_gamma);
    L.gamma1 = reinterpret_cast<const RsTab *>(base + p->off_gamma1);
    L.u = p->u.data();
    L.used = p->used.data();
    return in_scratch_slices(n, low_block_rows(p->C, k) * sb, s, [&](uint64_t s0, uint64_t cnt, uint8_t *scratch) {
      LowBlockArgs b = L;
      b.enc.data += s0 * ostride;
      b.rec += s0 * rstride;
      b.dec.out += s0 * outstride;
      b.enc.n_stripes = cnt;
      b.enc.scratch = scratch;
      return launch_low_blocks(b, s);
    });
  }
  const KernelChoice kc = choose_decode_w(p->W, sb, max_nv);
  const uint8_t *base = static_cast<const uint8_t *>(p->buf->p);
  const uint8_t *tw = static_cast<const uint8_t *>(p->tw->p);
  DecodeArgs a{};
  a.orig = orig;
  a.orig_stripe_stride = ostride;
  a.rec = rec;
  a.rec_stripe_stride = rstride;
  a.out = out;
  a.out_stripe_stride = outstride;
  a.shard_bytes = sb;
  a.tab_ifft = reinterpret_cast<const RsTab *>(tw);
  a.tab_fft = reinterpret_cast<const RsTab *>(tw + p->off_fft);
  a.tab_pre = reinterpret_cast<const RsTab *>(base);
  a.tab_post = a.tab_pre + p->W;
  a.pos_src = reinterpret_cast<const int32_t *>(base + 2ull * p->W * sizeof(RsTab));
  a.pos_dst = a.pos_src + p->W;
  a.work = p->W;
  a.trunc = p->trunc;
  a.trunc_fft = static_cast<uint32_t>(k);
  a.contig = kc.variant != Variant::kGeneric && contig_ok(sb, kc.nv);
  if (kc.variant != Variant::kGeneric) {
    a.n_stripes = n;
    HIP_TRY(launch_decode(kc, a, s));
    return RS_OK;
  }
  return in_scratch_slices(n, decode_generic_rows(p->W, p->trunc, k) * sb, s, [&](uint64_t s0, uint64_t cnt, uint8_t *scratch) {
    DecodeArgs b = a;
    b.orig += s0 * ostride;
    b.rec += s0 * rstride;
    b.out += s0 * outstride;
    b.n_stripes = cnt;
    b.scratch = scratch;
    b.scratch_stripes = cnt;
    return launch_decode(kc, b, s);
  });
}

int low_warm(int dev, uint64_t k, uint64_t m, uint64_t sb, const uint8_t *present) {
  std::shared_ptr<LowDecodePlan> p;
  if (int st = get_low_decode_plan(dev, k, m, sb, present, p)) return st;
  if (p->net) {
    queue_net(*p->net, sb);
    jit::wait_pending();
  }
  return RS_OK;
}

// ---- the low-rate reconstruct in block form (round 5). Decoding the residual codeword
// (received ^ the codeword of d' = the received originals with the erased ones zero) gives the
// erased originals; its only non-zero inputs are the syndromes s = rec ^ Enc(d') on the
// recovery rows R used (the first e present: exactly C positions are then known, the code's
// dimension; the other present rows join the erasures). Those rows sit in blocks K >= 1 of
// C positions; the outputs in block 0. Tracking the W-point decode block by block: the IFFT's
// layers below C are per-block IFFT_{C, skew KC}; its layers >= C, the derivative's bits >= C
// and the FFT's layers >= C only combine whole blocks with scalar factors, and the derivative's
// bits below C act inside a block (D_C). So block 0 after the FFT's top layers is
//   D_C(sum_K alpha_K b_K) + sum_K beta_K b_K,   b_K = IFFT_{C, skew KC}(L_R s_R in block K)
// and the erased original g is g^(65535 - e_g) FFT_{C, skew 0, trunc k}(that)_g. The scalars
// come from running the top layers' schedule on block coefficients (Generic.zig:15-147,
// root.zig:306-312); the host selftest checks the form against scalar_reconstruct_low.
namespace {
uint16_t gm(uint16_t x, uint16_t y) { return x && y ? mul16(x, tables().log[y]) : 0; }
uint16_t tw(uint64_t idx) {  // the element a butterfly at skew index idx multiplies by (0: XOR-only)
  const uint16_t l = idx < kModulus ? tables().skew[idx] : static_cast<uint16_t>(kModulus);
  return l == kModulus ? 0 : tables().exp[l];
}
}  // namespace

void low_block_coefs(uint64_t k, uint64_t m, std::vector<uint16_t> &alpha, std::vector<uint16_t> &beta) {
  const uint64_t C = ceil_pow2(k), W = ceil_pow2(C + m), nb = W / C;
  std::vector<std::vector<uint16_t>> lam(nb, std::vector<uint16_t>(nb, 0));
  for (uint64_t J = 0; J < nb; J++) lam[J][J] = 1;
  auto axpy = [&](std::vector<uint16_t> &y, uint16_t t, const std::vector<uint16_t> &x) {  // y ^= t x
    for (uint64_t K = 0; K < nb; K++) y[K] ^= gm(t, x[K]);
  };
  for (uint64_t d = C; d < W; d *= 2)  // IFFT layers >= C: y ^= x; x ^= t y (Generic.zig:171-192)
    for (uint64_t g = 0; g < W; g += 2 * d) {
      const uint16_t t = tw(g + d - 1);
      for (uint64_t i = g; i < g + d; i += C) {
        auto &x = lam[i / C], &y = lam[(i + d) / C];
        for (uint64_t K = 0; K < nb; K++) y[K] ^= x[K];
        axpy(x, t, y);
      }
    }
  // block J = D_C(P_J) + Q_J: the derivative's bits >= C add whole blocks (root.zig:306-312)
  std::vector<std::vector<uint16_t>> P = lam, Q(nb, std::vector<uint16_t>(nb, 0));
  for (uint64_t J = 0; J < nb; J++)
    for (uint64_t b = 1; b < nb; b <<= 1)
      if (!(J & b) && J + b < nb)
        for (uint64_t K = 0; K < nb; K++) Q[J][K] ^= lam[J + b][K];
  for (uint64_t d = W / 2; d >= C && d > 0; d /= 2)  // FFT layers >= C: x ^= t y; y ^= x (Generic.zig:149-169)
    for (uint64_t g = 0; g < W; g += 2 * d) {
      const uint16_t t = tw(g + d - 1);
      for (uint64_t i = g; i < g + d; i += C) {
        const uint64_t x = i / C, y = (i + d) / C;
        axpy(P[x], t, P[y]);
        axpy(Q[x], t, Q[y]);
        for (uint64_t K = 0; K < nb; K++) P[y][K] ^= P[x][K], Q[y][K] ^= Q[x][K];
      }
    }
  alpha = P[0];
  beta = Q[0];
}

// The block form on one symbol per position: data k (erased entries ignored), par m,
// present k + m; restores data[g] for every erased g. Returns false if fewer than k present.
bool scalar_reconstruct_low_blocks(uint16_t *data, const uint16_t *par, const uint8_t *present, uint64_t k,
                                   uint64_t m) {
  const uint64_t C = ceil_pow2(k), end = C + m, W = ceil_pow2(end), nb = W / C;
  uint64_t e = 0;
  for (uint64_t i = 0; i < k; i++) e += present[i] ? 0 : 1;
  std::vector<uint8_t> received(W, 0), inR(m, 0);
  for (uint64_t i = 0; i < k; i++) received[i] = present[i] ? 1 : 0;
  uint64_t nr = 0;
  for (uint64_t r = 0; r < m && nr < e; r++)
    if (present[k + r]) received[C + r] = inR[r] = 1, nr++;
  if (nr < e) return false;
  std::vector<uint16_t> er(kOrder);
  erasure_logs_low(received.data(), k, m, er.data());
  std::vector<uint16_t> alpha, beta;
  low_block_coefs(k, m, alpha, beta);
  std::vector<uint16_t> coef(C, 0), U(C, 0), V(C, 0), b(C);
  for (uint64_t i = 0; i < k; i++) coef[i] = present[i] ? data[i] : 0;
  scalar_ifft(coef.data(), C, k, 0, false);  // the low-rate encode of d' (scalar_encode_low)
  for (uint64_t K = 1; K < nb; K++) {
    bool any = false;
    for (uint64_t q = 0; q < C && (K - 1) * C + q < m; q++) any |= inR[(K - 1) * C + q] != 0;
    if (!any) continue;
    b = coef;
    scalar_fft(b.data(), C, std::min(C, m - (K - 1) * C), K * C, false);  // Enc(d') rows of block K
    for (uint64_t q = 0; q < C; q++) {
      const uint64_t r = (K - 1) * C + q;
      b[q] = r < m && inR[r] ? mul16(static_cast<uint16_t>(par[r] ^ b[q]), er[C + r]) : 0;
    }
    scalar_ifft(b.data(), C, C, K * C, false);
    for (uint64_t q = 0; q < C; q++) U[q] ^= gm(alpha[K], b[q]), V[q] ^= gm(beta[K], b[q]);
  }
  for (uint64_t q = 0; q < C; q++) {  // D_C, ascending (reads original values above)
    uint16_t z = U[q];
    for (uint64_t w = 1; w < C; w <<= 1)
      if (!(q & w)) z ^= U[q + w];
    V[q] ^= z;
  }
  scalar_fft(V.data(), C, k, 0, false);
  for (uint64_t g = 0; g < k; g++)
    if (!present[g]) data[g] = mul16(V[g], static_cast<uint16_t>(kModulus - er[g]));
  return true;
}

const char *low_encode_kernel_name(uint64_t k, uint64_t m, uint64_t sb) {
  if (map_net_ok(k, m, sb)) return net_name("encode_low", k, m);
  return choose_encode_low(ceil_pow2(k), sb, 4).name;
}

const char *low_reconstruct_kernel_name(uint64_t k, uint64_t m, uint64_t sb, uint64_t e) {
  if (map_net_ok(k, e, sb)) return net_name("reconstruct_low", k, e);
  if (block_form(k, m, sb, e)) return "low_blocks";  // get_low_decode_plan's predicate
  return choose_decode_w(ceil_pow2(ceil_pow2(k) + m), sb, 4).name;
}

}  // namespace host
}  // namespace rs

using namespace rs;
using namespace rs::host;

extern "C" int rs_lowrate_selftest(uint64_t k, uint64_t m, int trials, uint64_t seed, uint64_t *mismatches) {
  return guarded([&]() -> int {
    const int hr = use_high_rate(k, m);
    if (hr < 0) return fail(-hr, "unsupported shard count (root.zig:397-415)");
    if (hr == 1) return fail(RS_ERR_INVALID_ARGUMENT, "not a low-rate code");
    const uint64_t C = ceil_pow2(k), W = ceil_pow2(C + m);
    uint64_t state = seed * 0x9E3779B97F4A7C15ull + 1;
    auto rnd = [&]() {  // splitmix64
      uint64_t z = (state += 0x9E3779B97F4A7C15ull);
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      return z ^ (z >> 31);
    };
    uint64_t bad = 0;
    std::vector<uint16_t> data(k), par(m), sym(W), er(kOrder);
    std::vector<uint8_t> present(k + m), received(W);
    for (int t = 0; t < trials; t++) {
      for (auto &x : data) x = static_cast<uint16_t>(rnd());
      scalar_encode_low(data.data(), k, m, false, par.data());
      // lose e random originals (1..min(k, m)) and as many recovery shards as leaves >= k present
      const uint64_t e = 1 + rnd() % std::min(k, m);
      std::fill(present.begin(), present.end(), 1);
      for (uint64_t c = 0; c < e;) {
        const uint64_t i = rnd() % k;
        if (present[i]) present[i] = 0, c++;
      }
      const uint64_t drop = rnd() % (m - e + 1);
      for (uint64_t c = 0; c < drop;) {
        const uint64_t r = rnd() % m;
        if (present[k + r]) present[k + r] = 0, c++;
      }
      std::fill(received.begin(), received.end(), 0);
      std::fill(sym.begin(), sym.end(), 0);
      for (uint64_t i = 0; i < k; i++)
        if (present[i]) received[i] = 1, sym[i] = data[i];
      for (uint64_t r = 0; r < m; r++)
        if (present[k + r]) received[C + r] = 1, sym[C + r] = par[r];
      erasure_logs_low(received.data(), k, m, er.data());
      scalar_reconstruct_low(sym.data(), received.data(), er.data(), k, m);
      for (uint64_t i = 0; i < k; i++)
        if (!present[i] && sym[i] != data[i]) bad++;
      // the block form (syndromes of the first e present recovery rows, C-point transforms)
      if (W / C > kLowBlockMaxBlocks) continue;
      std::vector<uint16_t> blk = data;
      for (uint64_t i = 0; i < k; i++)
        if (!present[i]) blk[i] = static_cast<uint16_t>(rnd());
      if (!scalar_reconstruct_low_blocks(blk.data(), par.data(), present.data(), k, m)) bad++;
      for (uint64_t i = 0; i < k; i++)
        if (blk[i] != data[i]) bad++;
    }
    if (mismatches) *mismatches = bad;
    return RS_OK;
  });
}
