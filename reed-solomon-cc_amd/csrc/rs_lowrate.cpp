// rs_lowrate.cpp — the low-rate codec (§8 f4; the reference panics: root.zig:119-121, 226-228).
#include "rs_host.hpp"

namespace rs {
namespace host {

// ------------------------------------------------------- low-rate codec (§8 f4)
// The reference panics on low rate (root.zig:119-121, 226-228). Here the encode
// is reed-solomon-simd's low-rate encoder (rs_gf.hpp scalar_encode_low; parity
// unpinned: no reference output exists) and a reconstruct is the unique MDS
// solution, derived by linear algebra from the encode map. Both run as maps on
// the network kernels, or on the table matrix kernels in groups of <= 8 outputs.

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

int low_encode(int dev, uint64_t k, uint64_t m, uint64_t sb, uint64_t n, const uint8_t *orig, uint64_t ostride,
               uint8_t *rec, uint64_t rstride, uint32_t flags, int max_nv, hipStream_t s) {
  std::shared_ptr<MapPlan> lp;
  if (int st = get_low_encode_plan(dev, k, m, flags, lp)) return st;
  return run_map(*lp, sb, n, orig, ostride, nullptr, 0, rec, rstride, max_nv, s);
}

int low_reconstruct(int dev, uint64_t k, uint64_t m, uint64_t sb, uint64_t n, const uint8_t *present,
                    const uint8_t *orig, uint64_t ostride, const uint8_t *rec, uint64_t rstride, uint8_t *out,
                    uint64_t outstride, uint32_t flags, int max_nv, hipStream_t s) {
  std::shared_ptr<MapPlan> lp;
  if (int st = get_low_decode_plan(dev, k, m, flags, present, lp)) return st;
  return run_map(*lp, sb, n, orig, ostride, rec, rstride, out, outstride, max_nv, s);
}

const char *low_encode_kernel_name(uint64_t k, uint64_t m, uint64_t sb) {
  return map_net_ok(k, m, sb) ? net_name("encode_low", k, m) : "lowrate_matrix";
}

const char *low_reconstruct_kernel_name(uint64_t k, uint64_t m, uint64_t sb, uint64_t e) {
  return map_net_ok(k, e, sb) ? net_name("reconstruct_low", k, e) : "lowrate_matrix";
}

}  // namespace host
}  // namespace rs

using namespace rs;
using namespace rs::host;

