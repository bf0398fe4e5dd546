// rs_batch_dev.cpp — device-resident batches: rs_encode_batch_dev / rs_reconstruct_batch_dev
// (one erasure pattern per batch) and the shard-tail wrappers (root.zig:338-348).
#include "rs_host.hpp"

extern "C" int rs_encode_batch_dev(uint64_t, uint64_t, size_t, uint64_t, const void *, uint64_t, void *, uint64_t,
                                   uint32_t, rs_stream_t);
extern "C" int rs_reconstruct_batch_dev(uint64_t, uint64_t, size_t, uint64_t, const uint8_t *, const void *, uint64_t,
                                        const void *, uint64_t, void *, uint64_t, uint32_t, rs_stream_t);

namespace rs {
namespace host {

// ---------------------------------------------------------- shard tails
// Batches whose shard_bytes is not a multiple of 64 run on padded copies
// ([stripe][shard][ceil(sb/64)*64], tail chunk in the reference's layout) in
// slices of <= 1 GiB, then the outputs are unpadded.

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

int encode_tail(uint64_t k, uint64_t m, uint64_t sb, uint64_t n, const uint8_t *orig, uint64_t ostride, uint8_t *rec,
                uint64_t rstride, uint32_t flags, hipStream_t s) {
  const uint64_t psb = (sb + 63) / 64 * 64;
  const uint64_t cap = std::max<uint64_t>(1, std::min<uint64_t>(n, kTailSliceBytes / ((k + m) * psb)));
  void *buf = nullptr;
  HIP_TRY(dev_malloc_async(&buf, cap * (k + m) * psb, s));
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
  HIP_TRY(dev_malloc_async(&buf, cap * (k + m + e) * psb, s));
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

}  // namespace host
}  // namespace rs

using namespace rs;
using namespace rs::host;

extern "C" {

int rs_encode_batch_dev(uint64_t k, uint64_t m, size_t sb, uint64_t n_stripes, const void *d_original,
                        uint64_t orig_stride, void *d_recovery, uint64_t rec_stride, uint32_t flags,
                        rs_stream_t stream) {
  TraceScope ts;
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
    if (is_low_rate(k, m))
      return low_encode(dev, k, m, sb, n_stripes, static_cast<const uint8_t *>(d_original), orig_stride,
                        static_cast<uint8_t *>(d_recovery), rec_stride, flags, max_nv, s);
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
    HIP_TRY(dev_malloc_async(&scratch, per * plan->work * sb, s));
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
  TraceScope ts;
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
    if (is_low_rate(k, m))
      return low_reconstruct(dev, k, m, sb, n_stripes, present, static_cast<const uint8_t *>(d_original), orig_stride,
                             static_cast<const uint8_t *>(d_recovery), rec_stride, static_cast<uint8_t *>(d_restored),
                             out_stride, flags, max_nv, static_cast<hipStream_t>(stream));
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
    // the fused FFT reconstruct (wide codes): syndromes and decode in one kernel, the
    // pattern as data. RS_AMD_FDEC=auto runs it until a network compiled
    // for the pattern is loaded (as fast for the syndrome maps, faster for few losses)
    if (plan->fdec_blk && max_nv == 4 && fdec_supports(k, m, sb, flags)) {
      const jit::Kernel *nk = plan->net && fdec_mode() != 1 ? net_kernel(*plan->net, sb) : nullptr;
      if (!nk && plan->pdec && pdec_enabled()) {  // the pattern compiled in, once loaded
        const fftnet::Spec *pfs = nullptr;
        if (const jit::Kernel *pk = fft_kernel(*plan->pdec, sb, &pfs)) {
          HIP_TRY(fftnet::launch(*pk, *pfs, static_cast<const uint8_t *>(d_original ? d_original : d_recovery),
                                 orig_stride, static_cast<const uint8_t *>(d_recovery), rec_stride,
                                 static_cast<uint8_t *>(d_restored), out_stride, sb, n_stripes,
                                 static_cast<hipStream_t>(stream)));
          return RS_OK;
        }
      }
      if (!nk) {
        std::shared_ptr<WpsSlot> ws;
        wps_slot(dev, k, m, 0, ws);
        const fftnet::Spec *dfs = nullptr;
        if (const jit::Kernel *fk = fft_kernel(*ws->dec, sb, &dfs)) {
          HIP_TRY(fftnet::launch(*fk, *dfs, static_cast<const uint8_t *>(d_original ? d_original : d_recovery),
                                 orig_stride, static_cast<const uint8_t *>(d_recovery), rec_stride,
                                 static_cast<uint8_t *>(d_restored), out_stride, sb, n_stripes,
                                 static_cast<hipStream_t>(stream), static_cast<const uint32_t *>(plan->fdec_blk->p),
                                 plan->fdec_words, true));
          return RS_OK;
        }
        if (fdec_mode() == 1) return fail(RS_ERR_DEVICE, "RS_AMD_FDEC=1: fused FFT reconstruct kernel unavailable");
      }
    }
    if (plan->lite && (st = get_decode_plan(dev, k, m, sb, flags, present, plan, 1))) return st;
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
      // syndromes on the code's FFT kernel with the batch's mask block; the pattern's e x e
      // network once its background compile has landed, the generic solve until then
      // (DESIGN.md §3.3), the table kernels only without those
      const jit::Kernel *nk = plan->net && max_nv == 4 ? net_kernel(*plan->net, sb) : nullptr;
      const bool blk = plan->syn_blk && max_nv == 4;
      const jit::Kernel *dk = nullptr, *sk = nullptr;
      const fftnet::Spec *dfs = nullptr;
      if (blk) {
        std::shared_ptr<WpsSlot> ws;
        wps_slot(dev, k, m, 0, ws);
        dk = fft_kernel(*ws->fft, sb, &dfs);
        if (!nk && dk) sk = wps_solve_kernel(*ws);
      }
      // syndrome scratch in slices of <= 4 GiB (slices small enough for the 256 MB Infinity
      // Cache measured slower: less work per launch)
      const uint64_t cap = 4096ull << 20;
      const uint64_t per = std::max<uint64_t>(1, std::min<uint64_t>(n_stripes, cap / (m * sb)));
      void *scratch = nullptr;
      HIP_TRY(dev_malloc_async(&scratch, per * m * sb, s));
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
        const uint32_t *bk = blk ? static_cast<const uint32_t *>(plan->syn_blk->p) : nullptr;
        if (dk)
          err = fftnet::launch(*dk, *dfs, eb.data, orig_stride, nullptr, 0, eb.parity, m * sb, sb, cnt, s, bk,
                               plan->syn_pw, true);
        else
          err = launch_encode(ke, eb, s);
        if (err == hipSuccess) {
          if (nk)
            err = jit::launch(*nk, db.orig, orig_stride, db.rec, rec_stride, db.out, out_stride, sb, cnt, s, db.xsrc,
                              db.xsrc_stripe_stride);
          else if (sk)  // the e x e map is compiling: the generic solve on the same syndromes
            err = psyn::launch_solve(*sk, db.rec, rec_stride, db.xsrc, db.xsrc_stripe_stride, db.out, out_stride, sb,
                                     cnt, bk, plan->syn_pw, plan->syn_dmw, plan->syn_cs, s, true);
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
    // launch_decode_generic: the transform plus the FFT's kept rows, per stripe
    const uint64_t rows = decode_generic_rows(plan->work, a.trunc, a.trunc_fft);
    const uint64_t per = slice_stripes(n_stripes, rows * sb);
    void *scratch = nullptr;
    HIP_TRY(dev_malloc_async(&scratch, per * rows * sb, s));
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

// Drive one erasure pattern to its steady state: the plan the pattern's later calls use
// (a lite plan's background upgrade included) and every kernel they launch, compiled and
// loaded, blocking until done. The same sequence a stream of calls would go through
// (get_decode_plan's first and second use), without waiting for those calls.
int rs_reconstruct_warm(uint64_t k, uint64_t m, size_t sb, const uint8_t *present, uint32_t flags) {
  return guarded([&]() -> int {
    if (!present) return fail(RS_ERR_INVALID_ARGUMENT, "present == NULL");
    int st = check_codec(k, m, sb);
    if (st) return st;
    uint64_t have = 0, e = 0;
    for (uint64_t i = 0; i < k + m; i++) have += present[i] != 0;
    for (uint64_t i = 0; i < k; i++) e += present[i] == 0;
    if (have < k) return fail(RS_ERR_NOT_ENOUGH_SHARDS, "fewer than original_count shards present");
    if (e == 0) return RS_OK;
    const uint64_t psb = (sb + 63) / 64 * 64;  // tails run on padded shards
    int dev;
    if ((st = current_device(&dev))) return st;
    if (is_low_rate(k, m)) return low_warm(dev, k, m, psb, present);
    std::shared_ptr<DecodePlan> plan;
    if ((st = get_decode_plan(dev, k, m, psb, flags, present, plan))) return st;
    if (plan->lite) {  // a later use decides (and queues) the upgrade; wait for it
      if ((st = get_decode_plan(dev, k, m, psb, flags, present, plan, 3))) return st;
      jit::wait_pending();
      if ((st = get_decode_plan(dev, k, m, psb, flags, present, plan))) return st;
    }
    const fftnet::Spec *fs = nullptr;
    if (plan->inv_fft) (void)fft_kernel(*plan->inv_fft, psb, &fs);
    if (plan->net) queue_net(*plan->net, psb);
    // a build that spills is rebuilt with less prefetch (fftnet::get): a few rounds
    for (int i = 0; i < 4 && plan->pdec && !fft_kernel(*plan->pdec, psb, &fs); i++) jit::wait_pending();
    if (plan->fdec_blk && fdec_supports(k, m, psb, flags)) {
      std::shared_ptr<WpsSlot> ws;
      wps_slot(dev, k, m, 0, ws);
      (void)fft_kernel(*ws->dec, psb, &fs);
    }
    if (plan->syndrome && plan->syn_blk) {
      std::shared_ptr<WpsSlot> ws;
      wps_slot(dev, k, m, 0, ws);
      (void)fft_kernel(*ws->fft, psb, &fs);
      (void)wps_solve_kernel(*ws);
    }
    jit::wait_pending();
    return RS_OK;
  });
}

}  // extern "C"
