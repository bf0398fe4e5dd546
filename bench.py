#!/usr/bin/env python3
"""Headline benchmark: device-resident RS(10,4) encode + reconstruct, 1 MiB shards.

One step = encode a 4096-stripe batch (BASELINE configs[1]) + reconstruct the
4 erased data shards {0,1,2,3} of every stripe of that batch (configs[2]),
inputs resident in HBM. N GPUs (torchrun) = N independent stripe batches, one
per rank (configs[3]: 4096 stripes per GPU, weak scaling, no data-path
collective; the only collectives are the timing barrier and max).

value = user data processed by the step (k*shard_bytes per stripe for the
encode plus the same for the reconstruct) / step time, GiB/s, all ranks.
Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-cc_amd"))
import reedsol_amd as R  # noqa: E402  (after torch: one HIP runtime)
from reedsol_amd.sharding import all_ok, max_over_ranks  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--shard-bytes", type=int, default=1 << 20)
    ap.add_argument("--stripes", type=int, default=4096, help="stripes per GPU")
    ap.add_argument("--erase", type=str, default="0,1,2,3", help="erased original indices")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget for the CPU baseline leg (0 = skip)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--c4-reps", type=int, default=5,
                    help="BASELINE configs[4] (RS(200,55) 256 KiB x 512) GPU leg after the timed region, N=1 (0 = skip)")
    ap.add_argument("--c4-stripes", type=int, default=512, help="stripes of the configs[4] leg (SURVEY.md §8(d): 512)")
    return ap.parse_args()


def _threads():
    """Host threads for the CPU leg: the cores this process may run on, capped at the
    GPU box's CPU share (16 per GPU: the harness sizes worker pools to it; os.cpu_count()
    there reports the whole machine). The per-core rate is reported beside it."""
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    return max(1, min(int(os.environ.get("RS_BENCH_CPU_THREADS", "16")), cores)), cores


def _cpu_leg(O, k, m, sb, erase, n_stripes, threads, rng):
    """Oracle (C restatement of the reference engine, AVX2 pshufb) encode + reconstruct
    of n_stripes stripes: (GiB/s combined, encode GiB/s, reconstruct GiB/s)."""
    present = np.ones(k + m, np.uint8)
    present[erase] = 0
    data = rng.integers(0, 256, (n_stripes, k, sb), dtype=np.uint8)
    t0 = time.perf_counter()
    par = O.encode_batch(k, m, data, threads=threads)
    t1 = time.perf_counter()
    O.reconstruct_batch(k, m, present, np.concatenate([data, par], axis=1), threads=threads)
    t2 = time.perf_counter()
    gib = k * sb * n_stripes / 2**30
    return 2 * gib / (t2 - t0), gib / (t1 - t0), gib / (t2 - t1)


def cpu_baseline(k, m, sb, erase, budget_s):
    """Oracle on the host cores: the same step (encode + reconstruct) on a bounded
    stripe sample, single-threaded and on `threads` cores; plus the other BASELINE
    configs (c0: RS(4,2) 64 KiB, benchmarks.zig:25-60 protocol; c4: RS(200,55) 256 KiB
    losing 55 data shards) and the reference harness shapes."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    threads, cores = _threads()
    rng = np.random.default_rng(7)
    # calibrate on one stripe single-threaded, then size both legs to the budget
    per_stripe = 2 * k * sb / 2**30 / _cpu_leg(O, k, m, sb, erase, 1, 1, rng)[0]
    n1 = max(1, min(32, int(budget_s * 0.25 / per_stripe)))
    v1, e1, r1 = _cpu_leg(O, k, m, sb, erase, n1, 1, rng)
    nt = max(threads, min(64, int(budget_s * 0.45 / per_stripe * threads)))
    vt, et, rt = _cpu_leg(O, k, m, sb, erase, nt, threads, rng)
    # c4: RS(200,55) 256 KiB, 55 erased data shards (every third), threads stripes
    c4_erase = list(range(1, 200, 3))[:55]
    v4, e4, r4 = _cpu_leg(O, 200, 55, 256 << 10, c4_erase, threads, threads, rng)
    _, e41, r41 = _cpu_leg(O, 200, 55, 256 << 10, c4_erase, 1, 1, rng)
    return {
        "value": round(vt, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": f"RS({k},{m}) {sb >> 10} KiB shards, {nt} stripes encode + reconstruct {len(erase)} erased, "
                  f"{threads} threads of {cores} visible (oracle/rs_oracle.c AVX2 engine)",
        "single_thread": {"value": round(v1, 3), "cores": 1, "encode_GiBps": round(e1, 3),
                          "reconstruct_GiBps": round(r1, 3), "sample_stripes": n1},
        "per_core_GiBps": round(vt / threads, 3),
        "encode_GiBps": round(et, 3),
        "reconstruct_GiBps": round(rt, 3),
        "per_config": {
            "c0 RS(4,2) 64KiB 1 stripe insert+encode us (benchmarks.zig protocol, 1 thread)":
                round(O.bench_encode_ns(4, 2, 64 << 10, 500) / 1e3, 3),
            "c1/c2 RS(10,4) 1MiB encode+reconstruct4 GiB/s": round(vt, 3),
            "c4 RS(200,55) 256KiB encode GiB/s": round(e4, 3),
            "c4 RS(200,55) 256KiB reconstruct55 GiB/s": round(r4, 3),
            "c4 sample": f"{threads} stripes, {threads} threads",
            "c4 RS(200,55) 256KiB encode GiB/s 1 thread": round(e41, 3),
            "c4 RS(200,55) 256KiB reconstruct55 GiB/s 1 thread": round(r41, 3),
        },
        "harness": harness_protocol(O),
        "cpu_model": _cpu_model(),
    }


def verify_parity(k, m, data, parity, stripes=(0, -1)):
    """Checker, outside the timed region: the GPU parity of a few whole stripes against
    the oracle (C restatement of the reference, oracle/rs_oracle.c)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    idx = sorted({s % data.shape[0] for s in stripes})
    d = data[idx].cpu().numpy()
    got = parity[idx].cpu().numpy()
    return bool((O.encode_batch(k, m, d, threads=_threads()[0]) == got).all())


def harness_protocol(O, iters=2000):
    """The reference's own benchmark (benchmarks.zig:11-60): mean microseconds per
    single-threaded insert + encode of (32,32) and (64,64) at 1 KiB shards, random
    bytes, timed natively in the oracle (rso_bench_encode, AVX2 engine)."""
    return {f"encode:{k}/{m} 1KiB us": round(O.bench_encode_ns(k, m, 1024, iters) / 1e3, 3)
            for k, m in ((32, 32), (64, 64))}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _time_calls(fn, reps):
    """HIP events around `reps` calls (after one untimed call) and the kernels every call
    launched (rs_last_kernels: what ran, not what a name query predicts)."""
    fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ran = set()
    a.record()
    for _ in range(reps):
        fn()
        ran.add(";".join(R.last_kernels()))
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps, sorted(ran)


def c4_leg(dev, reps, n=512):
    """BASELINE configs[4] on the GPU, outside the timed region (rank 0, N=1): RS(200,55)
    256 KiB x n (512 stripes, 25 GiB of data) encode and reconstruct of 55
    erased data shards (every third from 1), HIP events over `reps` calls.

    reconstruct: the pattern's steady state after rs_reconstruct_warm (its full plan and
    every kernel it launches compiled and loaded); reconstruct_fused / reconstruct_network:
    the two forms a wide-code pattern can run (RS_AMD_FDEC=1: the fused FFT reconstruct;
    RS_AMD_FDEC=0: syndromes on the FFT kernel + the pattern's e x e network), each warmed
    the same way. Every entry names the kernels its calls actually launched. Then a cold
    pattern (every third from 2, never seen by the process): its first calls without any
    warm-up, as a repair service meeting a new pattern runs them. Restored shards are
    checked against the data."""
    k, m, sb = 200, 55, 256 << 10
    lost = list(range(1, k, 3))[:m]
    present = [0 if i in lost else 1 for i in range(k)] + [1] * m
    g = torch.Generator(device=dev)
    g.manual_seed(0xC4)
    data = torch.randint(0, 256, (n, k, sb), dtype=torch.uint8, device=dev, generator=g)
    par = torch.empty((n, m, sb), dtype=torch.uint8, device=dev)
    out = torch.empty((n, m, sb), dtype=torch.uint8, device=dev)
    R.encode_batch_dev(k, m, data, par)
    torch.cuda.synchronize()
    R.net_wait()
    res = {"workload": f"RS(200,55) 256 KiB shards x {n} stripes; reconstruct: 55 erased data shards "
                       "(every third from 1)"}
    alg = (k + m) * sb * n
    ok = True

    def entry(ms, ran):
        return {"ms": round(ms, 3), "GiBps": round(k * sb * n / (ms * 1e-3) / 2**30, 1),
                "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4), "kernels": ran}

    res["encode"] = entry(*_time_calls(lambda: R.encode_batch_dev(k, m, data, par), reps))
    rec = lambda: R.reconstruct_batch_dev(k, m, present, data, par, out)  # noqa: E731
    prev = os.environ.get("RS_AMD_FDEC")
    try:
        for name, fdec in (("reconstruct", prev), ("reconstruct_fused", "1"), ("reconstruct_network", "0")):
            if fdec is None:
                os.environ.pop("RS_AMD_FDEC", None)
            else:
                os.environ["RS_AMD_FDEC"] = fdec
            R.reconstruct_warm(k, m, sb, present)
            out.zero_()
            res[name] = entry(*_time_calls(rec, reps))
            ok = ok and bool(torch.equal(out, data[:, lost]))
    finally:
        if prev is None:
            os.environ.pop("RS_AMD_FDEC", None)
        else:
            os.environ["RS_AMD_FDEC"] = prev
    res["verified"] = ok
    # cold pattern: first calls of an erasure pattern whose kernels are not compiled
    lost_c = list(range(2, k, 3))[:m]
    present_c = [0 if i in lost_c else 1 for i in range(k)] + [1] * m
    calls = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        a.record()
        R.reconstruct_batch_dev(k, m, present_c, data, par, out)
        ran = R.last_kernels()
        b.record()
        torch.cuda.synchronize()
        calls.append({"wall_ms": round((time.perf_counter() - t0) * 1e3, 3), "gpu_ms": round(a.elapsed_time(b), 3),
                      "kernels": ran})
    res["reconstruct_cold"] = {"calls": calls, "pattern": "55 erased data shards, every third from 2",
                               "note": "first calls of a new pattern, no warm-up (plan build included in wall_ms)",
                               "verified": bool(torch.equal(out, data[:, lost_c]))}
    R.net_wait()  # the cold pattern's queued upgrade finishes here, not during process exit
    del data, par, out
    torch.cuda.empty_cache()
    return res


def load_traffic(kernel_names):
    """HBM bytes per launch from the committed PMC summary (profiles/traffic.json),
    written by tools/pmc_traffic.py from separate rocprofv3 --pmc passes."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None
    try:
        t = json.load(open(path))
    except (OSError, ValueError):
        return None
    return {n: t[n] for n in kernel_names if n in t}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # local % count: identical on a full node; lets a rehearsal put 2 ranks on 1 GPU
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # nccl (= RCCL) on the node; RS_BENCH_BACKEND=gloo rehearses N>1 on one GPU
        backend = os.environ.get("RS_BENCH_BACKEND", "nccl")
        dist.init_process_group(backend, device_id=dev if backend == "nccl" else None)
    k, m, sb, n = args.k, args.m, args.shard_bytes, args.stripes
    erase = [int(x) for x in args.erase.split(",") if x != ""]
    e = len(erase)
    present = [0 if i in erase else 1 for i in range(k)] + [1] * m

    # synthetic, distinct per rank; resident in HBM before timing
    g = torch.Generator(device=dev)
    g.manual_seed(0x5EED0000 + rank)
    data = torch.randint(0, 256, (n, k, sb), dtype=torch.uint8, device=dev, generator=g)
    parity = torch.empty((n, m, sb), dtype=torch.uint8, device=dev)
    restored = torch.empty((n, e, sb), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()

    launched = {"encode": set(), "reconstruct": set()}  # rs_last_kernels after every call

    def step(ev=None):
        if ev:
            ev[0].record(stream)
        R.encode_batch_dev(k, m, data, parity, stream=stream)
        launched["encode"].add(";".join(R.last_kernels()))
        if ev:
            ev[1].record(stream)
        R.reconstruct_batch_dev(k, m, present, data, parity, restored, stream=stream)
        launched["reconstruct"].add(";".join(R.last_kernels()))
        if ev:
            ev[2].record(stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    for v in launched.values():
        v.clear()  # report what the timed steps ran
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(events[i])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = time.perf_counter() - t0
    enc_ms = float(np.mean([ev[0].elapsed_time(ev[1]) for ev in events]))
    rec_ms = float(np.mean([ev[1].elapsed_time(ev[2]) for ev in events]))
    t = max_over_ranks(t, device=dev)  # slowest rank sets the step time
    enc_ms = max_over_ranks(enc_ms, device=dev)
    rec_ms = max_over_ranks(rec_ms, device=dev)

    ok = None
    if not args.no_verify:  # restored == erased data, and 2 whole stripes' parity == the oracle's
        ok = all_ok(bool(torch.equal(restored, data[:, erase])) and verify_parity(k, m, data, parity), device=dev)

    if rank == 0:
        data_bytes = k * sb * n  # per rank per op
        gib = 2 * data_bytes * world * args.steps / t / 2**30
        enc_alg = (k + m) * sb * n  # algorithmic HBM bytes per encode launch
        rec_alg = (k + e) * sb * n  # k received shards read + e restored written
        kinds = {"encode": (enc_ms, enc_alg, R.encode_kernel_name(k, m, sb)),
                 "reconstruct": (rec_ms, rec_alg, R.reconstruct_kernel_name(k, m, sb, present))}
        dom = max(kinds, key=lambda x: kinds[x][0])
        ms, alg, kname = kinds[dom]
        achieved = alg / (ms * 1e-3) / 1e9
        traffic = load_traffic([kname]) or {}
        tr = traffic.get(kname)
        roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBPS, 4),
                    # HBM bytes per launch from PMC (profiles/traffic.json, per stripe x this batch)
                    "traffic": int(tr["hbm_bytes_per_stripe"] * n) if tr else None,
                    "traffic_source": (tr["method"] + "; " + tr["workload"] +
                                       ("" if tr.get("stripes_per_launch") == n else
                                        f"; scaled per stripe to {n} stripes")) if tr else None,
                    "kernel": kname, "algorithmic_bytes_per_launch": alg, "avg_launch_ms": round(ms, 4),
                    "per_kernel": {kk: {"kernel": v[2], "avg_ms": round(v[0], 4),
                                        "achieved_GBps": round(v[1] / (v[0] * 1e-3) / 1e9, 1),
                                        "frac": round(v[1] / (v[0] * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                                        "data_GiBps": round(data_bytes / (v[0] * 1e-3) / 2**30, 1),
                                        "launched": sorted(launched[kk])}
                                   for kk, v in kinds.items()}}
        cpu = None  # host-core baseline: rank 0 at N=1 only (the driver's N>1 runs skip it)
        if args.cpu_seconds > 0 and world == 1:
            cpu = cpu_baseline(k, m, sb, erase, args.cpu_seconds)
        c4 = None  # configs[4] on the GPU (not part of `value`)
        if args.c4_reps > 0 and world == 1:
            del data, parity, restored
            torch.cuda.empty_cache()
            try:
                c4 = c4_leg(dev, args.c4_reps, args.c4_stripes)
            except Exception as ex:  # never costs the headline line
                c4 = {"error": str(ex)[:200]}
        out = {
            "metric": "device-resident encode+reconstruct GiB/s per GPU (RS(10,4), 1 MiB shards); % HBM roofline",
            "value": round(gib, 2),
            "value_per_gpu": round(gib / world, 2),
            "value_note": "value = user data encoded + reconstructed by all GPUs per second (whole job); "
                          "value_per_gpu = value / n_gpus",
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (torch.randint bytes, resident in HBM)",
            "config": {"workload": f"RS({k},{m}) {sb >> 10} KiB shards, {n}-stripe batch per GPU: encode + "
                                   f"reconstruct {e} erased data shards {erase}",
                       "k": k, "m": m, "shard_bytes": sb, "stripes_per_gpu": n, "erased": erase,
                       "parallelism": f"stripe-sharded x{world} (no data-path collective)"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "encode_GiBps": round(data_bytes * world / (enc_ms * 1e-3) / 2**30, 2),
            "reconstruct_GiBps": round(data_bytes * world / (rec_ms * 1e-3) / 2**30, 2),
            "verified": ok,
            "verified_how": "restored shards == erased data on every stripe; parity of stripes 0 and n-1 == oracle",
            "c4_gpu": c4,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
