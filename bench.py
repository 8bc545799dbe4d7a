#!/usr/bin/env python3
"""Throughput benchmark of the ns-nnsp hot path on MI355X.

Metric (BASELINE.json): audio frames/s (16 kHz, 10 ms hop) per node at
1/2/4/8 GPUs, bit-exact vs the reference.  One frame = 160 samples of one
stream.  The default workload is BASELINE configs[4], the one the 1/2/4/8-GPU
curve is quoted on: the full VAD -> Hi-Galaxy KWS -> S2I cascade
(nnCntrlClass_exec per frame) with 32768 streams per GPU (262144 on 8 GPUs).
--net vad|kws|s2i runs configs[1..3] (one net, 8192 streams/GPU).

A "step" is one chunk of --frames frames (default 100 = 1 s of audio) for
every stream of the GPU's shard; streams carry their state across steps
(continuous audio).  Input PCM is generated on the device (SplitMix64,
oracle.synthetic_pcm) before the timed region; nothing crosses PCIe inside it.

Multi-GPU: one process per GPU (torch.distributed, RCCL backend); every rank
owns its own shard of --streams streams (weak scaling, no data-path
collective); value = all frames of all ranks / max over ranks of the timed
wall time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# algorithmic work per frame (denominators of roofline.achieved)
FE_MULS_PER_FRAME = 5912           # integer multiplies of one front-end frame
NN_MACS_PER_INFERENCE = {"vad": 14616, "kws": 56448, "s2i": 72072}
FE_HBM_BYTES_PER_FRAME = 320 + 80  # PCM in + normalised features out (cascade: + 80, int32 log-Mel out)

WORKLOADS = {  # BASELINE.json configs
    "cascade": "configs[4]: VAD->Hi-Galaxy KWS->S2I cascade, 32768 streams/GPU (262144 on 8 GPUs)",
    "vad": "configs[1]: VAD net, 8192 streams/GPU, Mel front end + int8xint16 FC/LSTM, 64b accum",
    "kws": "configs[2]: Hi-Galaxy KWS net, 8192 streams/GPU",
    "s2i": "configs[3]: S2I RNN, 8192 streams/GPU",
}


def cpu_baseline(net: str, acc32: bool, seconds: float = 1.5, procs: int | None = None) -> dict:
    """Oracle ("port") timed on the host cores, one process per core (the
    reference library is not re-entrant, so the reference scales by processes)."""
    import multiprocessing as mp

    procs = procs or min(16, os.cpu_count() or 1)
    with mp.get_context("fork").Pool(procs) as pool:
        t0 = time.perf_counter()
        res = pool.starmap(_cpu_worker, [(net, acc32, seconds, i) for i in range(procs)])
        wall = time.perf_counter() - t0
    frames = sum(res)
    return {"value": frames / wall, "unit": "frames/s", "cores": procs, "kind": "port",
            "sample": f"{procs} processes x ~{seconds:.1f} s of continuous synthetic streams "
                      f"(32 streams x 100-frame chunks each), {net} net, "
                      f"{'32' if acc32 else '64'}b accumulator; C oracle -O3"}


def _cpu_worker(net: str, acc32: bool, seconds: float, idx: int) -> int:
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import OracleCascade, OracleNet, synthetic_pcm

    from nnsp_amd.nets import synth_net

    S, T = 32, 100
    if net == "cascade":
        orc = OracleCascade({n: OracleNet(synth_net(n), acc32=acc32) for n in ("vad", "kws", "s2i")})
        st = orc.new_states(S)
        run = lambda pcm: orc.run(pcm, st)  # noqa: E731
    else:
        orc = OracleNet(synth_net(net), acc32=acc32)
        st = orc.new_states(S)
        run = lambda pcm: orc.run(pcm, st, want_logits=False, want_feats=False)  # noqa: E731
    frames, t0, c = 0, time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds:
        run(synthetic_pcm(S, T, s0=idx * S, t0=c * T))
        frames += S * T
        c += 1
    return frames


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--net", default="cascade", choices=sorted(WORKLOADS))
    ap.add_argument("--streams", type=int, default=0,
                    help="streams per GPU (default 32768 for the cascade, 8192 for one net)")
    ap.add_argument("--window", type=int, default=-1, help="cascade frames per round (-1: library default)")
    ap.add_argument("--frames", type=int, default=100, help="frames per step (chunk)")
    ap.add_argument("--acc32", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=1.5)
    ap.add_argument("--profile-json", default=os.path.join(ROOT, "profiles", "pmc_latest.json"))
    args = ap.parse_args()

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)

    from nnsp_amd import _lib
    from nnsp_amd.engine import NNSPBatch, device_info

    _lib.check(_lib.lib().nnsp_set_device(local if world > 1 else 0), "set_device")
    S = args.streams or (32768 if args.net == "cascade" else 8192)
    T, K, W = args.frames, args.steps, args.warmup
    cascade = args.net == "cascade"
    if cascade:
        from nnsp_amd.engine import NNSPCascade

        nets = {n: NNSPBatch(n, S, T, acc32=args.acc32) for n in ("vad", "kws", "s2i")}
        eng = NNSPCascade(nets)
        if args.window >= 0:
            eng.set_window(args.window)
    else:
        eng = NNSPBatch(args.net, S, T, acc32=args.acc32)
    # inputs resident in HBM before timing: one chunk buffer per step
    bufs = [torch.empty((S, T, 160), dtype=torch.int16, device="cuda") for _ in range(W + K)]
    for i, b in enumerate(bufs):
        _lib.check(_lib.lib().nnsp_synth_pcm(b.data_ptr(), S, T, 0x4E4E5350, rank * S, i * T, 4096,
                                             eng.stream), "synth_pcm")
    trig = torch.empty((S, T), dtype=torch.int16, device="cuda")
    out3 = torch.empty((S, T, 3), dtype=torch.int16, device="cuda")

    def step(buf):
        if cascade:   # per frame: the NNSP_ID that ran, its trigger and outputs
            eng.exec_device(buf.data_ptr(), T, None, trig.data_ptr(), out3.data_ptr())
        else:
            eng.exec_device(buf.data_ptr(), T, trig.data_ptr())

    eng.sync()
    torch.cuda.synchronize()
    for i in range(W):
        step(bufs[i])
    eng.sync()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    kt = {}            # kernel -> total ms over the timed steps
    kframes = {}       # kernel -> frames (fe) or NN frames it processed
    klaunch = {}       # kernel -> launches
    rounds = 0
    t0 = time.perf_counter()
    for i in range(K):
        step(bufs[W + i])
        if cascade:
            r, _, _ = eng.last_stats()
            rounds += r
            kt["fe_kernel"] = kt.get("fe_kernel", 0.0) + eng.fe_stats()   # shared log-Mel, one launch
            kframes["fe_kernel"] = kframes.get("fe_kernel", 0) + S * T
            klaunch["fe_kernel"] = klaunch.get("fe_kernel", 0) + 1
            for n in ("vad", "kws", "s2i"):
                f, _, _, nl = eng.net_stats(n)   # per-net device times: instrumented step below
                kframes[f"nn_{n}"] = kframes.get(f"nn_{n}", 0) + f
                klaunch[f"nn_{n}"] = klaunch.get(f"nn_{n}", 0) + nl
        else:
            f, n = eng.last_timing()   # syncs the stream: per-step kernel times
            kt["fe_kernel"] = kt.get("fe_kernel", 0.0) + f
            kt[f"nn_{args.net}"] = kt.get(f"nn_{args.net}", 0.0) + n
            kframes["fe_kernel"] = kframes.get("fe_kernel", 0) + S * T
            kframes[f"nn_{args.net}"] = kframes.get(f"nn_{args.net}", 0) + S * T
            klaunch["fe_kernel"] = klaunch.get("fe_kernel", 0) + 1
            klaunch[f"nn_{args.net}"] = klaunch.get(f"nn_{args.net}", 0) + 1
    eng.sync()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    net_ms = {}
    if cascade:
        # per-net device time per round (HIP events around each net's work):
        # one extra, untimed chunk with the events on -- they cost a few
        # percent, so the timed steps run without them.  The nets run
        # concurrently on three streams: these spans overlap.
        eng.set_timing(True)
        step(bufs[W + K - 1])
        eng.sync()
        eng.set_timing(False)
        rl, rfe, rnn = eng.round_stats()
        net_ms["rounds"] = {"streams_listed": rl.tolist(),
                            "cold_fe_ms": [[round(float(x), 4) for x in r] for r in rfe],
                            "nn_ms": [[round(float(x), 4) for x in r] for r in rnn],
                            "net_order": ["s2i", "vad", "kws"]}
        for n in ("vad", "kws", "s2i"):
            f, fe, nn, nl = eng.net_stats(n)
            net_ms[n] = {"cold_fe_ms": fe, "nn_ms": nn, "frames": f, "rounds": nl}
    frames = S * T * K * world
    value = frames / elapsed

    if rank == 0:
        info = device_info()
        cu, clk = info["compute_units"], info["clock_khz"] * 1e3
        valu_peak = cu * 128 * clk / 1e12          # VALU lane-ops/s (4 SIMDs x 32 lanes per clock per CU)
        # integer multiplies issue at about half the add rate on gfx950: the
        # front end's ceiling is the measured v_mul_hi_i32 rate on all CUs
        # (profiles/microbench/valu_rates.hip, run on MI355X), scaled to this device
        mul_peak, mul_src = valu_peak * 0.5, "half the VALU lane-op rate (no probe file)"
        try:
            with open(os.path.join(ROOT, "profiles", "microbench", "valu_rates_mi355x.json")) as f:
                vr = json.load(f)
            mul_peak = vr["rates"]["v_mul_hi_i32"] / 1e12 * (cu * clk) / (vr["compute_units"] * vr["clock_khz"] * 1e3)
            mul_src = "measured v_mul_hi_i32 issue rate, profiles/microbench/valu_rates_mi355x.json"
        except Exception:
            pass
        mfma_peak = 5000.0                         # dense int8 MFMA Tops/s (MI355X_MICROARCH.md: 2x BF16 2.5 PF)
        # dominant kernel by device time.  In the cascade the nets' segment
        # kernels run concurrently on three streams, so their event spans are
        # not kernel durations; the one-launch shared front end is the largest
        # kernel there (profiles/*/kernel_stats.csv)
        dom = "fe_kernel" if cascade else max(kt, key=kt.get)
        launches = klaunch[dom]
        avg_launch_s = kt[dom] / 1e3 / launches    # HIP-event time on the engine's stream
        units = kframes[dom] / launches            # frames per launch
        if dom == "fe_kernel":
            per_unit = FE_MULS_PER_FRAME
            work = "integer multiplies (SURVEY 8(d): 5912 per frame) x frames per launch"
            peak, bound = mul_peak, "valu"
        else:
            n = dom[3:]
            per_unit = NN_MACS_PER_INFERENCE[n]    # one inference per 2 frames, 2 ops per MAC
            work = f"{n} int8xint16 MACs x2 ops x inferences (frames/2) per launch"
            peak, bound = mfma_peak, "mfma"
        achieved = units * per_unit / avg_launch_s / 1e12
        traffic = None
        try:
            with open(args.profile_json) as f:
                pj = json.load(f)
            if pj.get("workload") == args.net and pj.get("streams") == S and pj.get("frames") == T:
                traffic = pj["kernels"][dom]["hbm_bytes_per_launch"]
        except Exception:
            pass
        fe_s = kt["fe_kernel"] / 1e3
        out = {
            "metric": "audio frames/sec (16 kHz, 10 ms hop) per node; bit-exact vs ref",
            "value": value,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed / K * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32 (int16 PCM, q31 FFT, int8xint16 MACs)",
            "data": "synthetic SplitMix64 int16 PCM generated on device; seeded synthetic weights of the reference net shapes",
            "config": {"workload": WORKLOADS[args.net], "net": args.net, "streams_per_gpu": S,
                       "frames_per_step": T, "accumulator": "32b" if args.acc32 else "64b",
                       "parallelism": f"stream shards x{world}"},
            "kernels_ms_per_step": {k: v / K for k, v in kt.items()},
            **({"nets_one_chunk": net_ms} if cascade else {}),
            "frames_scheduled_per_step": {k: v // K for k, v in kframes.items()},
            "roofline": {"kernel": dom, "bound": bound,
                         "achieved": achieved, "peak": peak, "unit": "Tops/s",
                         "frac": achieved / peak, "work": work,
                         "peak_source": mul_src if dom == "fe_kernel" else "dense int8 MFMA (MI355X_MICROARCH.md)",
                         "valu_lane_peak": valu_peak,
                         "traffic": traffic, "traffic_unit": "HBM bytes per launch (PMC, profiles/)",
                         "launches_per_step": launches / K, "avg_launch_ms": avg_launch_s * 1e3,
                         "frames_per_launch": units,
                         "hbm_achieved_GBps": kframes["fe_kernel"] * (FE_HBM_BYTES_PER_FRAME + (80 if cascade else 0))
                         / fe_s / 1e9,
                         "hbm_peak_GBps": 8000.0},
            "device": info,
        }
        if cascade:
            out["cascade"] = {"rounds_per_step": rounds / K,
                              "speculation_overhead": sum(kframes[f"nn_{n}"] for n in ("vad", "kws", "s2i"))
                              / (S * T * K) - 1.0}
        if not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.net, args.acc32, args.cpu_seconds)
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
