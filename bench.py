#!/usr/bin/env python3
"""Throughput benchmark of the ns-nnsp hot path on MI355X.

Metric (BASELINE.json): audio frames/s (16 kHz, 10 ms hop) per node, bit-exact
vs the reference.  One frame = 160 samples of one stream.  A "step" is one
chunk of --frames frames (default 100 = 1 s of audio) for every stream of the
GPU's shard; streams carry their state across steps (continuous audio).  Input
PCM is generated on the device (SplitMix64, oracle.synthetic_pcm) before the
timed region; nothing crosses PCIe inside it.

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
FE_HBM_BYTES_PER_FRAME = 320 + 80  # PCM in + normalised features out

WORKLOADS = {  # BASELINE.json configs
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
    from oracle import OracleNet, synthetic_pcm

    from nnsp_amd.nets import synth_net

    orc = OracleNet(synth_net(net), acc32=acc32)
    S, T = 32, 100
    st = orc.new_states(S)
    frames, t0, c = 0, time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds:
        pcm = synthetic_pcm(S, T, s0=idx * S, t0=c * T)
        orc.run(pcm, st, want_logits=False, want_feats=False)
        frames += S * T
        c += 1
    return frames


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--net", default="vad", choices=sorted(WORKLOADS))
    ap.add_argument("--streams", type=int, default=8192, help="streams per GPU")
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
    S, T, K, W = args.streams, args.frames, args.steps, args.warmup
    eng = NNSPBatch(args.net, S, T, acc32=args.acc32)
    # inputs resident in HBM before timing: one chunk buffer per step
    bufs = [torch.empty((S, T, 160), dtype=torch.int16, device="cuda") for _ in range(W + K)]
    for i, b in enumerate(bufs):
        _lib.check(_lib.lib().nnsp_synth_pcm(b.data_ptr(), S, T, 0x4E4E5350, rank * S, i * T, 4096,
                                             eng.stream), "synth_pcm")
    trig = torch.empty((S, T), dtype=torch.int16, device="cuda")
    eng.sync()
    torch.cuda.synchronize()
    for i in range(W):
        eng.exec_device(bufs[i].data_ptr(), T, trig.data_ptr())
    eng.sync()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    fe_ms = nn_ms = 0.0
    t0 = time.perf_counter()
    for i in range(K):
        eng.exec_device(bufs[W + i].data_ptr(), T, trig.data_ptr())
        f, n = eng.last_timing()   # syncs the stream: per-step kernel times
        fe_ms += f
        nn_ms += n
    eng.sync()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    frames = S * T * K * world
    value = frames / elapsed

    if rank == 0:
        info = device_info()
        # dominant kernel: the front end (VALU-bound integer work)
        fe_avg_s = fe_ms / K / 1e3
        nn_avg_s = nn_ms / K / 1e3
        dom = "fe_kernel" if fe_avg_s >= nn_avg_s else "nn_kernel"
        cu, clk = info["compute_units"], info["clock_khz"] * 1e3
        valu_peak = cu * 128 * clk / 1e12          # int32 VALU lane-ops/s (4 SIMD32 per CU)
        if dom == "fe_kernel":
            achieved = S * T * FE_MULS_PER_FRAME / fe_avg_s / 1e12
        else:
            achieved = S * T / 2 * NN_MACS_PER_INFERENCE[args.net] * 2 / nn_avg_s / 1e12
        traffic = None
        try:
            with open(args.profile_json) as f:
                pj = json.load(f)
            if pj.get("net") == args.net and pj.get("streams") == S and pj.get("frames") == T:
                traffic = pj.get("fe_kernel_hbm_bytes_per_launch")
        except Exception:
            pass
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
            "kernels_ms_per_step": {"fe_kernel": fe_ms / K, "nn_kernel": nn_ms / K},
            "roofline": {"kernel": dom, "bound": "valu",
                         "achieved": achieved, "peak": valu_peak, "unit": "Tops/s",
                         "frac": achieved / valu_peak,
                         "work": ("integer multiplies (SURVEY 8(d): 5912 per frame)" if dom == "fe_kernel"
                                  else "int8xint16 MAC x2 ops"),
                         "traffic": traffic,
                         "hbm_achieved_GBps": S * T * FE_HBM_BYTES_PER_FRAME / fe_avg_s / 1e9,
                         "hbm_peak_GBps": 8000.0},
            "device": info,
        }
        if not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args.net, args.acc32, args.cpu_seconds)
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
