// rs_plans.cpp — per-(k, m, flags) encode plans and per-erasure-pattern reconstruct
// plans: butterfly tables, GF(2) maps for the bit-sliced networks, the syndrome
// map, FFT-kernel specs; and the plan-time compile checks of the C ABI.
#include "rs_host.hpp"

namespace rs {
namespace host {

PlanCache<EncodePlan> g_enc_plans;
PlanCache<DecodePlan> g_dec_plans;

void release_plans() {
  std::lock_guard<std::mutex> lk(g_plan_mu);
  g_enc_plans.clear();
  g_dec_plans.clear();
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
// the unique restored data does not depend on which k). Under D1, and under D2 where
// it drops a chunk, the literal reconstruct is no decoder of the parity, so its output
// depends on every present shard: keep ALL of them then, exactly as the reference would
// receive them (literal_decode).
void reconstruct_map(uint64_t k, uint64_t m, uint32_t flags, const uint8_t *present, jit::NetSpec &ns) {
  const bool d1 = flags & RS_FLAG_QUIRK_D1;
  const uint64_t C = ceil_pow2(m), W = ceil_pow2(C + k);
  uint64_t present_count = 0;
  for (uint64_t i = 0; i < k + m; i++) present_count += present[i] ? 1 : 0;
  const uint64_t want = literal_decode(k, m, flags) ? present_count : k;
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
  alloc_point();
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

// The syndrome path's plan block (rs_host.hpp DecodePlan::syn_blk), the layout of the
// per-stripe k_wps_plan blocks: fftnet::dyn mask words (erased data positions, then the
// rows R stored), then at word dmw: [0] restored outputs, [1] e, [2 + i] = R_i,
// [66 + i * cs + j] = A^-1[j][i] in polynomial form (from the syndrome map's blocks:
// the image of the symbol 1 = the coefficient in Cantor coordinates).
int syndrome_block(int dev, uint64_t k, uint64_t m, const uint8_t *present, const jit::NetSpec &map,
                        DecodePlan &plan) {
  fftnet::Spec fs;
  fs.k = static_cast<uint32_t>(k);
  fs.m = static_cast<uint32_t>(m);
  fs.dyn = true;
  const uint32_t e = map.n_out, dmw = fftnet::dyn_mask_words(fs), cs = wps_coef_stride(e);
  const uint32_t pw = dmw + 2 + 64 + 64 * cs;
  std::vector<uint32_t> blk(pw, 0);
  for (uint64_t i = 0; i < k; i++)
    if (!present[i]) blk[i / 32] |= 1u << (i % 32);
  const uint16_t *cantor = cantor_basis();
  for (uint32_t i = 0; i < e; i++) {
    const uint32_t r = static_cast<uint32_t>(map.src[i] & kSrcIndexMask);
    blk[dmw - 2 + r / 32] |= 1u << (r % 32);
    blk[dmw + 2 + i] = r;
    for (uint32_t j = 0; j < e; j++) {
      const uint16_t c = map.images[(static_cast<size_t>(i) * e + j) * 16];
      uint32_t poly = 0;
      for (int b = 0; b < 16; b++) poly ^= (c >> b & 1) ? cantor[b] : 0u;
      blk[dmw + 2 + 64 + i * cs + j] = poly;
    }
  }
  blk[dmw] = e;
  blk[dmw + 1] = e;
  if (int st = upload(blk.data(), blk.size() * sizeof(uint32_t), dev, plan.syn_blk)) return st;
  plan.syn_dmw = dmw;
  plan.syn_pw = pw;
  plan.syn_cs = cs;
  return RS_OK;
}

// root.zig:268-335 erasure pattern -> evalPoly -> masks and table block (FFT
// kernels), or -> the reconstruct's linear map as an e x k matrix (matrix kernel).
int get_decode_plan(int dev, uint64_t k, uint64_t m, uint64_t sb, uint32_t flags, const uint8_t *present,
                    std::shared_ptr<DecodePlan> &out, int how) {
  const bool full = how == 1;
  const std::string mode = decode_mode_env();
  std::string key = std::to_string(dev) + "/" + std::to_string(k) + "/" + std::to_string(m) + "/" +
                    std::to_string(flags) + "/" + mode + "/" + std::to_string(sb % 512 == 0) + "/" +
                    std::to_string(jit::enabled() && jit::shard_ok(sb)) + "/" +
                    std::to_string(fft_enabled() && fftnet::supports(k, m, sb)) + "/" +
                    std::to_string(jit::max_blocks()) + "/" + std::to_string(jit::max_async_blocks()) + "/" +
                    std::to_string(fdec_mode()) + "/" + std::to_string(fdec_supports(k, m, sb, flags)) + "/" +
                    std::to_string(pdec_enabled()) + "/";
  key.reserve(key.size() + k + m);
  for (uint64_t i = 0; i < k + m; i++) key.push_back(present[i] ? '1' : '0');
  std::shared_ptr<DecodePlan> lite;
  {
    std::lock_guard<std::mutex> lk(g_plan_mu);
    if ((out = g_dec_plans.find(key))) {
      if (!out->lite) return RS_OK;
      if (!full && fdec_mode() == 1) return RS_OK;  // forced fused form: the block is all it needs
      if (how == 0) out->uses++;
      lite = out;  // a later use: build the full plan (network, tables) now if one is worth it
      out.reset();
    }
  }
  const bool d1 = flags & RS_FLAG_QUIRK_D1;
  const uint64_t C = ceil_pow2(m), end = C + k, W = ceil_pow2(C + k);
  uint64_t e = 0, present_count = 0;
  for (uint64_t i = 0; i < k; i++) e += present[i] ? 0 : 1;
  for (uint64_t i = 0; i < k + m; i++) present_count += present[i] ? 1 : 0;
  // first use of a wide-code pattern: only the fused FFT reconstruct's block
  const bool every_lost = e == k && present_count == m;  // the inverse form's case stays on the full plan
  if (!lite && !full && e > 0 && !every_lost && m <= 64 && fdec_supports(k, m, sb, flags) &&
      (mode == "auto" || mode == "net")) {
    alloc_point();
    auto plan = std::make_shared<DecodePlan>();
    fftnet::Spec ds;
    ds.k = static_cast<uint32_t>(k);
    ds.m = static_cast<uint32_t>(m);
    ds.dyn = ds.decode = true;
    std::vector<uint32_t> blk(fftnet::decode_block_words(ds));
    if (fftnet::decode_block(ds, present, blk.data()) == RS_OK) {
      if (int st = upload(blk.data(), blk.size() * sizeof(uint32_t), dev, plan->fdec_blk)) return st;
      plan->fdec_words = static_cast<uint32_t>(blk.size());
      plan->lite = true;
      plan->e = static_cast<uint32_t>(e);
      std::lock_guard<std::mutex> lk(g_plan_mu);
      out = g_dec_plans.insert(key, plan);
      return RS_OK;
    }
  }
  int kind = decode_kind(k, m, flags, e, present_count, sb);
  // bit-sliced network (rs_jit.hpp): the same e x k map as the matrix kernels at a
  // fraction of their VALU cost, so preferred whenever it applies (modes auto / net)
  const uint64_t n_in_want = literal_decode(k, m, flags) ? present_count : k;
  const bool use_net = (mode == "auto" || mode == "net") && jit::enabled() &&
                       jit::supports(static_cast<uint32_t>(n_in_want), static_cast<uint32_t>(e), sb);
  if (use_net && kind == 0) kind = e <= kMatrixMaxOut ? 1 : 2;  // table kernels stay as the fallback
  // past the synchronous cap: the same map compiled in the background, the matrix
  // kernel meanwhile (RS(200,55) losing 8: 400 blocks, against syndrome + encode)
  const bool use_net_async = !use_net && kind != 0 && direct_net_async(e, n_in_want, sb, mode, k, m, flags);
  // a lite plan stays lite unless a network would beat the fused kernel: a direct map
  // (few losses: RS(200,55) 256 KiB x 256 losing 8, 2.6 vs 4.5 ms) or the syndrome path's
  // e x e map for e >= 3/4 m (55 losses 6.6 vs 6.9 ms; 20 losses the fused kernel wins, 4.9
  // vs 6.2 ms; profiles/r03/fdec/). The others skip the host plan algebra (10-40 ms) and
  // the background compile for good.
  // a reused wide-code pattern gets the fused kernel with the pattern compiled in (constant
  // locator multiplies: no scalar-loaded masks); it replaces the syndrome
  // path's e x e network, and a direct network (few losses) stays ahead of it. k <= 256: the
  // compile grows with the code (RS(200,55) 8-16 s, RS(1000,64) 45 s of hipRTC per pattern)
  // Only one steady-state kernel per pattern: a direct network (few losses) or this one
  // (queuing both cost a compile whose kernel never ran). Per-pattern compiles are
  // bounded (rs_host.hpp pdec_after / RS_AMD_PDEC_MAX / pdec_queue): a pattern seen fewer
  // times, past its code's budget, or while the worker is backed up keeps the fused kernel
  // with the pattern as data (a later use retries the last two).
  const bool pdec_want = e > 0 && !every_lost && m <= 64 && k <= kPdecMaxK && pdec_enabled() &&
                         fdec_supports(k, m, sb, flags) && (mode == "auto" || mode == "net") && !use_net &&
                         !use_net_async;
  const bool syn_wins = !pdec_want && syndrome_pick(k, m, e, flags, sb, mode) && 4 * e >= 3 * m;
  if (lite && how != 2 && !full && pdec_want && !use_net && !use_net_async && !syn_wins &&
      (lite->upgrading.load() ||
       (how == 0 && (lite->uses.load() < pdec_after() || jit::pending_jobs() > pdec_queue())) ||
       !pdec_admit(dev, k, m, key))) {
    out = lite;  // not (yet) worth a compile, or already queued
    return RS_OK;
  }
  // how == 1 (a call the fused kernels cannot serve, e.g. max_nv != 4) takes the same reuse
  // gate: a pattern below RS_AMD_PDEC_AFTER uses spends none of the code's RS_AMD_PDEC_MAX
  // budget on a kernel that call cannot launch
  const bool pdec_on = pdec_want && (how != 1 || (lite && lite->uses.load() >= pdec_after())) &&
                       pdec_admit(dev, k, m, key);
  if (lite && !full && !use_net && !use_net_async && !syn_wins && !pdec_on) {
    out = lite;
    return RS_OK;
  }
  if (lite && (how == 0 || how == 3)) {  // the full plan is built on the worker; the fused kernel meanwhile
    out = lite;
    if (!lite->upgrading.exchange(true)) {
      std::vector<uint8_t> pres(present, present + k + m);
      // the job also queues the full plan's network compile (behind it on the worker, so
      // rs_net_wait returns only once the pattern's steady-state kernel is loaded)
      if (!jit::run_host_job("plan:" + key, [dev, k, m, sb, flags, pres] {
            std::shared_ptr<DecodePlan> p;
            if (get_decode_plan(dev, k, m, sb, flags, pres.data(), p, 2) != RS_OK || !p) return;
            if (p->net) queue_net(*p->net, sb);
            if (p->pdec) {  // compiled here, on the worker (a build that spills is rebuilt with
              // less prefetch at once, not at the pattern's next call); the slot's async lookup
              // then finds it in the module cache
              fftnet::Spec ps = p->pdec->spec;
              std::string err;
              bool pending = false;
              (void)fftnet::get(ps, false, err, pending);
            }
          }))
        lite->upgrading = false;
    }
    return RS_OK;
  }
  const bool use_syn = !use_net && !use_net_async && !pdec_on && syndrome_pick(k, m, e, flags, sb, mode);
  if (use_syn) kind = e <= kMatrixMaxOut ? 1 : 2;
  // the syndromes' e x e map as a network too (its table kernel stays the fallback)
  const bool syn_net = use_syn && (mode == "auto" || mode == "net" || mode == "syndrome") && jit::enabled() &&
                       jit::supports_async(static_cast<uint32_t>(e), static_cast<uint32_t>(e), sb);
  const bool use_matrix = kind != 0;

  alloc_point();
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

  if (pdec_on) {
    plan->pdec = std::make_shared<FftSlot>();
    plan->pdec->async = true;
    fftnet::Spec &ps = plan->pdec->spec;
    ps.k = static_cast<uint32_t>(k);
    ps.m = static_cast<uint32_t>(m);
    ps.decode = true;
    ps.present.assign(present, present + k + m);
  }
  // the fused FFT reconstruct's block for this pattern (wide codes): the
  // form every pattern runs until a network compiled for it is loaded
  if (lite) {
    plan->fdec_blk = lite->fdec_blk;
    plan->fdec_words = lite->fdec_words;
  } else if (e > 0 && m <= 64 && fdec_supports(k, m, sb, flags)) {
    fftnet::Spec ds;
    ds.k = static_cast<uint32_t>(k);
    ds.m = static_cast<uint32_t>(m);
    ds.dyn = ds.decode = true;
    std::vector<uint32_t> blk(fftnet::decode_block_words(ds));
    if (fftnet::decode_block(ds, present, blk.data()) == RS_OK) {
      if (int st = upload(blk.data(), blk.size() * sizeof(uint32_t), dev, plan->fdec_blk)) return st;
      plan->fdec_words = static_cast<uint32_t>(blk.size());
    }
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
      // Enc(d') on the code's FFT kernel with the batch's mask block (Spec::dyn: erased data
      // read as zero, only the rows R stored): compiled once per code, as fast as a kernel
      // specialised for the pattern (RS(200,55) losing 55: 6.59 vs 6.62 ms for the whole
      // reconstruct, profiles/r03/synform.log), so no per-pattern FFT compile
      if (fft_enabled() && fftnet::supports(k, m, sb) && fftnet::pieces(sb) == 1 && sb % jit::kUnitBytes == 0 &&
          m <= 64)
        if ((st = syndrome_block(dev, k, m, present, map, *plan))) return st;
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
      if (lite) plan->net->uses = 1;  // the lite plan's call was the pattern's first use
      plan->net->spec = std::move(map);
    }
    plan->e = static_cast<uint32_t>(n_out);
    plan->n_in = static_cast<uint32_t>(n_in);
    plan->off_mat = 0;
    plan->off_src = tabs.size() * sizeof(RsTab);
    std::lock_guard<std::mutex> lk(g_plan_mu);
    out = lite ? g_dec_plans.replace(key, plan) : g_dec_plans.insert(key, plan);
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
  out = lite ? g_dec_plans.replace(key, plan) : g_dec_plans.insert(key, plan);
  return RS_OK;
}

}  // namespace host
}  // namespace rs

using namespace rs;
using namespace rs::host;

extern "C" {

int rs_psyn_compile_check(uint64_t k, uint64_t m, uint32_t flags, double *compile_ms, uint64_t *code_bytes) {
  return guarded([&]() -> int {
    int st = check_codec(k, m, jit::kUnitBytes);
    if (st) return st;
    if (is_low_rate(k, m) || (flags & RS_FLAG_QUIRK_D1))
      return fail(RS_ERR_INVALID_ARGUMENT, "no per-stripe syndrome network for this code");
    if (!psyn::supports(k, m, jit::kUnitBytes)) {
      if (!fftnet::supports(k, m, jit::kUnitBytes, true))
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
    if (!fftnet::supports(k, m, fftnet::kUnitBytes, true)) return fail(RS_ERR_INVALID_ARGUMENT, "no FFT kernel form");
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
    if (!fftnet::supports(k, m, fftnet::kUnitBytes, true)) return fail(RS_ERR_INVALID_ARGUMENT, "no FFT kernel form");
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

int rs_fft_decode_compile_check(uint64_t k, uint64_t m, double *compile_ms, uint64_t *code_bytes) {
  return guarded([&]() -> int {
    int st = check_codec(k, m, fftnet::kUnitBytes);
    if (st) return st;
    if (!fftnet::supports(k, m, fftnet::kUnitBytes, true)) return fail(RS_ERR_INVALID_ARGUMENT, "no FFT kernel form");
    fftnet::Spec spec;
    spec.k = static_cast<uint32_t>(k);
    spec.m = static_cast<uint32_t>(m);
    spec.dyn = spec.decode = true;
    std::string err;
    size_t bytes = 0;
    if (!fftnet::compile_check(spec, err, compile_ms, &bytes)) return fail(RS_ERR_DEVICE, err);
    if (code_bytes) *code_bytes = bytes;
    return RS_OK;
  });
}

int rs_fft_pdecode_compile_check(uint64_t k, uint64_t m, const uint8_t *present, double *compile_ms,
                                 uint64_t *code_bytes) {
  return guarded([&]() -> int {
    int st = check_codec(k, m, fftnet::kUnitBytes);
    if (st) return st;
    if (!present) return fail(RS_ERR_INVALID_ARGUMENT, "present == NULL");
    if (!fftnet::supports(k, m, fftnet::kUnitBytes, true)) return fail(RS_ERR_INVALID_ARGUMENT, "no FFT kernel form");
    uint64_t e = 0, have = 0;
    for (uint64_t i = 0; i < k; i++) e += present[i] ? 0 : 1;
    for (uint64_t i = 0; i < m; i++) have += present[k + i] ? 1 : 0;
    if (have < e) return fail(RS_ERR_NOT_ENOUGH_SHARDS, "fewer than original_count shards present");
    if (e == 0) return fail(RS_ERR_INVALID_ARGUMENT, "nothing erased");
    fftnet::Spec spec;
    spec.k = static_cast<uint32_t>(k);
    spec.m = static_cast<uint32_t>(m);
    spec.decode = true;
    spec.present.assign(present, present + k + m);
    std::string err;
    size_t bytes = 0;
    if (!fftnet::compile_check(spec, err, compile_ms, &bytes)) return fail(RS_ERR_DEVICE, err);
    if (code_bytes) *code_bytes = bytes;
    return RS_OK;
  });
}

int rs_debug_fft_stamps(uint64_t *out, uint64_t n) {
  return guarded([&]() -> int {
    if (!out) return fail(RS_ERR_INVALID_ARGUMENT, "out == NULL");
    return fftnet::read_stamps(out, n) == 0 ? RS_OK : fail(RS_ERR_DEVICE, "stamp buffer unavailable");
  });
}

int rs_fft_decode_selftest(uint64_t k, uint64_t m, uint32_t e, int trials, uint64_t *mismatches) {
  return guarded([&]() -> int {
    int st = check_codec(k, m, fftnet::kUnitBytes);
    if (st) return st;
    if (!fftnet::supports(k, m, fftnet::kUnitBytes, true) || e > m || e > k || e == 0)
      return fail(RS_ERR_INVALID_ARGUMENT, "no FFT decode form");
    const uint64_t bad = fftnet::decode_selftest(static_cast<uint32_t>(k), static_cast<uint32_t>(m), e, trials);
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

}  // extern "C"
