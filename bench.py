#!/usr/bin/env python3
"""Throughput benchmark of the ns-nnsp hot path on MI355X.

Metric (BASELINE.json): audio frames/s (16 kHz, 10 ms hop) per node at
1/2/4/8 GPUs, bit-exact vs the reference.  One frame = 160 samples of one
stream.  The default workload is BASELINE configs[4], the one the 1/2/4/8-GPU
curve is quoted on: the full VAD -> Hi-Galaxy KWS -> S2I cascade
(nnCntrlClass_exec per frame, evb/src/nnCntrlClass.c:152-272) with 32768
streams per GPU (262144 on 8 GPUs).  --net vad|kws|s2i runs configs[1..3] (one
net, 8192 streams/GPU).

Nets: the reference's own three nets (--weights ref, default: the def_nn*.c
tables, tests/golden/ref_nets.npz); --weights synth uses seeded synthetic
weights of the same shapes (a stress case: they trigger several times per
second on noise, so the cascade switches nets far more often).

Input: SplitMix64 int16 noise in [-4096, 4095] per stream;
every 4th stream instead replays python/test_wavs/{speech,galaxy,galaxy_s2i}.wav
(tests/golden/test_wavs.npz) cyclically from offset (s*1601) mod 160000
(--input noise: noise only).  Generated on the device before the timed region;
nothing crosses PCIe inside it.

A "step" is one chunk of --frames frames (default 100 = 1 s of audio) for
every stream of the GPU's shard; streams carry their state across steps
(continuous audio).

Multi-GPU: one process per GPU, launched by torch.distributed.run; a process
group is initialised whenever torch.distributed.run launched the process
(world size 1 included) -- gloo by default (--dist-backend), because it only
holds the barriers around the timed region and the timing / frame-count
reductions (an RCCL group shares HIP's hardware queues with the cascade's
streams: ~10 % slower).  Rank r owns a contiguous stream shard
(nnsp_amd.shard.shard_streams; weak scaling: --streams per GPU, strong:
--total-streams split), no data-path collective; value = frames of all ranks /
max over ranks of the timed wall time.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from nnsp_amd.shard import dist_env, reduce_run, shard_streams  # noqa: E402

# algorithmic work per frame (denominators of roofline.achieved)
FE_MULS_PER_FRAME = 5912           # integer multiplies of one front-end frame
NN_MACS_PER_INFERENCE = {"vad": 14616, "kws": 56448, "s2i": 72072}
FE_HBM_BYTES_PER_FRAME = 320 + 80  # PCM in + normalised features out (single net)
# cascade shared front end: PCM in, each of the three nets' normalised ring
# (3 x 80 B) out, and the look-back history of the next chunk (the chunk's
# last H = max look-back + 1 = 81 frames of PCM, stored once per chunk)
CASCADE_HIST_FRAMES = 81


def fe_bytes_per_frame(cascade: bool, T: int) -> float:
    if not cascade:
        return FE_HBM_BYTES_PER_FRAME
    return 320 + 3 * 80 + 320 * min(CASCADE_HIST_FRAMES, T) / T
# NN per inference (one per 2 frames): the 2 new context frames in (cascade:
# int32 log-Mel, 2 x 160 B) + per-frame outputs of its 2 frames (net, trigger,
# outputs[3]: 2 x 9 B)
NN_HBM_BYTES_PER_INFERENCE = 2 * 160 + 2 * 9
SEED = 0x4E4E5350
AMP = 4096
STRONG_TOTAL = 262144              # BASELINE configs[4]: streams per node

WORKLOADS = {  # BASELINE.json configs
    "cascade": "configs[4]: VAD->Hi-Galaxy KWS->S2I cascade, 32768 streams/GPU (262144 on 8 GPUs)",
    "vad": "configs[1]: VAD net, 8192 streams/GPU, Mel front end + int8xint16 FC/LSTM, 64b accum",
    "kws": "configs[2]: Hi-Galaxy KWS net, 8192 streams/GPU",
    "s2i": "configs[3]: S2I RNN, 8192 streams/GPU",
}


# ---------------------------------------------------------------------------
# CPU baseline: the oracle ("port"), one process per usable core
# ---------------------------------------------------------------------------
def host_cpu() -> dict:
    """The host's CPU share, each limit recorded on its own: the affinity mask,
    the cgroup v2 quota and the job-size variables the box exports; ``usable``
    is the smallest of them."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    host = os.cpu_count() or 1
    affinity = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else host
    cgroup = None
    try:   # cgroup v2 CPU quota: the share of the host this job may use
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()
            if q != "max":
                cgroup = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    env = {k: int(os.environ[k]) for k in ("OMP_NUM_THREADS", "MAX_JOBS") if os.environ.get(k, "").isdigit()}
    usable = min([affinity] + ([cgroup] if cgroup else []) + list(env.values()))
    return {"model": model, "host_cores": host, "affinity_cores": affinity, "cgroup_quota": cgroup,
            "env_quota": env, "usable_cores": usable}


def native_oracle() -> tuple[str | None, str]:
    """Compile the oracle -O3 -march=native for the host it runs on (SURVEY
    8(d)); the prebuilt -O3 build is the fallback."""
    src = os.path.join(ROOT, "oracle", "nnsp_oracle.c")
    out = os.path.join(tempfile.mkdtemp(prefix="nnsp_oracle_"), "liboracle_native.so")
    try:
        subprocess.run(["gcc", "-O3", "-march=native", "-fwrapv", "-fPIC", "-shared", "-o", out, src],
                       check=True, capture_output=True, timeout=120)
        return out, "gcc -O3 -march=native -fwrapv"
    except Exception:
        return None, "prebuilt oracle/liboracle.so (-O3; gcc -march=native build unavailable)"


def cpu_pool():
    """The CPU-baseline worker processes, forked before this process touches
    the GPU (a fork of a process holding a HIP context is unsafe); they idle
    until the GPU legs are done."""
    import multiprocessing as mp

    cpu = host_cpu()
    cpu["lib"], cpu["build"] = native_oracle()   # gcc runs before the GPU is touched too
    return mp.get_context("fork").Pool(cpu["usable_cores"]), cpu


def cpu_baseline(pool, cpu: dict, net: str, acc32: bool, weights: str, mix: bool, seconds: float,
                 portable: bool = False) -> dict:
    """The C oracle timed on the host cores, one process per core (the
    reference library keeps global scratch and is not re-entrant, so it scales
    by processes -- SURVEY 8(d))."""
    procs, lib = cpu["usable_cores"], cpu["lib"]
    res = pool.starmap(_cpu_worker, [(net, acc32, weights, mix, seconds, i, lib, portable) for i in range(procs)])
    rate = sum(f / t for f, t in res)   # the processes run concurrently: their rates add
    return {"value": rate, "unit": "frames/s", "cores": procs, "kind": "port",
            "cpu_model": cpu["model"], "host_cores": cpu["host_cores"], "affinity_cores": cpu["affinity_cores"],
            "cgroup_quota": cpu["cgroup_quota"], "env_quota": cpu["env_quota"],
            "build": cpu["build"],
            "sample": f"{procs} concurrent processes x ~{seconds:.0f} s each of 32 continuous streams in 100-frame "
                      f"chunks (the bench's input mix and weights, inputs generated before the timed loop), "
                      f"{net}, {'32' if acc32 else '64'}b accumulator"
                      f"{', the ARM_OPTIMIZED=0 build' if portable else ''}; value = sum of per-process frames / timed s"}


def _cpu_worker(net: str, acc32: bool, weights: str, mix: bool, seconds: float, idx: int,
                lib: str | None, portable: bool = False) -> tuple[int, float]:
    if lib:
        os.environ["NNSP_ORACLE_LIB"] = lib
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import OracleCascade, OracleNet, load_wavs, synthetic_pcm

    from nnsp_amd.nets import get_net

    wavs = load_wavs() if mix else None
    S, T, NC = 32, 100, 16
    if net == "cascade":
        orc = OracleCascade({n: OracleNet(get_net(n, weights), acc32=acc32, portable=portable, fe_portable=portable)
                             for n in ("vad", "kws", "s2i")})
        st = orc.new_states(S)
        run = lambda pcm: orc.run(pcm, st)  # noqa: E731
    else:
        orc = OracleNet(get_net(net, weights), acc32=acc32, portable=portable, fe_portable=portable)
        st = orc.new_states(S)
        run = lambda pcm: orc.run(pcm, st, want_logits=False, want_feats=False)  # noqa: E731
    chunks = [synthetic_pcm(S, T, SEED, t0=c * T, s0=idx * S, amp=AMP, wavs=wavs) for c in range(NC)]
    frames, c = 0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        run(chunks[c % NC])
        frames += S * T
        c += 1
    return frames, time.perf_counter() - t0


def dropin_cpu_baseline(net: str, pcm, lib: str | None) -> dict:
    """cpu_baseline leg of --dropin-latency: one stream of the same frames
    through the oracle on one core (its NNSPClass_exec path, frame after frame
    inside one C call: no per-frame Python in the timed loop)."""
    if lib:
        os.environ["NNSP_ORACLE_LIB"] = lib
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import OracleNet

    from nnsp_amd.nets import get_net

    orc = OracleNet(get_net(net, "ref"))
    st = orc.new_states(1)
    orc.run(pcm[None, :50], st, want_logits=False, want_feats=False)   # warm
    reps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 2.0:
        orc.run(pcm[None], st, want_logits=False, want_feats=False)
        reps += 1
    us = (time.perf_counter() - t0) / (reps * len(pcm)) * 1e6
    return {"us_per_frame": us, "cores": 1, "kind": "port",
            "sample": f"1 stream x {len(pcm)} frames of the speech wav, {reps} passes, one C call per pass"}


def dropin_latency(args, lib: str | None, build: str | None) -> dict:
    """The drop-in API's single-stream cost: the
    reference's NNSPClass_exec (nn_speech.c:74-127) called frame by frame on
    one stream, as an unchanged single-stream application calls it
    (nnCntrlClass.c:183).  Each call is one GPU batch of one stream: the frame
    goes up, the front end, the NN and the post-processing run, the result
    comes back.  Wall time per call, after warm-up."""
    import ctypes as C

    import numpy as np

    from nnsp_amd import _lib
    from nnsp_amd.nets import NN_ID, THRESH_CNTS, THRESH_PROB, get_net

    L = _lib.lib()
    z = np.load(os.path.join(ROOT, "tests", "golden", "test_wavs.npz"))
    T = 1000
    pcm = np.ascontiguousarray(z["speech"][:T * 160].reshape(T, 160), np.int16)
    out = {}
    for net in ("vad", "kws", "s2i"):
        h = _lib.NetHandle(get_net(net, "ref"))
        thr, cnt = np.array([THRESH_PROB], np.int16), np.array([THRESH_CNTS], np.int16)
        feat, inst = _lib.FeatureClass(), _lib.NNSPClass()
        _lib.check(L.NNSPClass_init(C.byref(inst), C.c_void_p(h.addr), C.byref(feat), bytes([NN_ID[net]]),
                                    _lib.ptr(h.mean), _lib.ptr(h.stdR), _lib.ptr(thr), _lib.ptr(cnt)), "init")
        L.NNSPClass_reset(C.byref(inst))
        frames = [np.ascontiguousarray(pcm[t]) for t in range(T)]
        for t in range(50):   # warm-up: weight image upload, kernel first launches
            L.NNSPClass_exec(C.byref(inst), _lib.ptr(frames[t]))
        dt = np.zeros(T)
        for t in range(T):
            t0 = time.perf_counter()
            L.NNSPClass_exec(C.byref(inst), _lib.ptr(frames[t]))
            dt[t] = time.perf_counter() - t0
        assert L.nnsp_legacy_status() == 0
        us = dt * 1e6
        e = {"gpu_us_per_frame_median": float(np.median(us)), "gpu_us_per_frame_p99": float(np.percentile(us, 99)),
             "gpu_us_per_frame_mean": float(us.mean()), "frames": T}
        if not args.no_cpu_baseline:
            e["cpu_baseline"] = dropin_cpu_baseline(net, pcm, lib)
            e["cpu_baseline"]["build"] = build
            e["gpu_over_cpu_time"] = e["gpu_us_per_frame_median"] / e["cpu_baseline"]["us_per_frame"]
        out[net] = e
    return out


# ---------------------------------------------------------------------------
# GPU run
# ---------------------------------------------------------------------------
def make_engine(net: str, S: int, T: int, acc32: bool, weights: str, window: int, arm_optimized: bool = True):
    from nnsp_amd.engine import NNSPBatch, NNSPCascade
    from nnsp_amd.nets import get_net

    if net == "cascade":
        nets = {n: NNSPBatch(get_net(n, weights), S, T, acc32=acc32, arm_optimized=arm_optimized)
                for n in ("vad", "kws", "s2i")}
        eng = NNSPCascade(nets)
        if window >= 0:
            eng.set_window(window)
        return eng
    return NNSPBatch(get_net(net, weights), S, T, acc32=acc32, arm_optimized=arm_optimized)


def chunk_step(eng, cascade: bool, T: int, buf, nxt, ran, trig, out3, lookahead: bool = True) -> None:
    """One timed step: a T-frame chunk of every stream (device buffers).  The
    cascade writes per frame the NNSP_ID that ran, its trigger and outputs, and
    the next chunk's front end runs ahead, overlapped with this chunk's nets
    (tests/test_gpu_benchloop.py runs this same function for parity)."""
    if cascade:
        eng.exec_device(buf.data_ptr(), T, ran.data_ptr(), trig.data_ptr(), out3.data_ptr(),
                        next_ptr=nxt.data_ptr() if (nxt is not None and lookahead) else None, next_T=T)
    else:
        eng.exec_device(buf.data_ptr(), T, trig.data_ptr())


def run_workload(args, S: int, s0: int, weights: str, dist=None) -> dict:
    """Create, warm up and time one workload on this rank's shard."""
    import numpy as np
    import torch

    from nnsp_amd import _lib

    T, K, W = args.frames, args.steps, args.warmup
    cascade = args.net == "cascade"
    eng = make_engine(args.net, S, T, args.acc32, weights, args.window, args.build == "shipped")
    dwav = None
    if args.input == "mix":
        z = np.load(os.path.join(ROOT, "tests", "golden", "test_wavs.npz"))
        wav = np.stack([z[k] for k in ("speech", "galaxy", "galaxy_s2i")])
        dwav = torch.from_numpy(wav).to("cuda")
    # inputs resident in HBM before timing: one chunk buffer per step (+1:
    # the chunk the last step's look-ahead front end reads)
    bufs = [torch.empty((S, T, 160), dtype=torch.int16, device="cuda") for _ in range(W + K + 1)]
    for i, b in enumerate(bufs):
        _lib.check(_lib.lib().nnsp_synth_pcm_mix(b.data_ptr(), S, T, SEED, s0, i * T, AMP,
                                                 dwav.data_ptr() if dwav is not None else None,
                                                 3 if dwav is not None else 0, 160000, 4, eng.stream), "synth_pcm")
    trig = torch.empty((S, T), dtype=torch.int16, device="cuda")
    out3 = torch.empty((S, T, 3), dtype=torch.int16, device="cuda")
    ran = torch.empty((S, T), dtype=torch.int8, device="cuda")

    def step(buf, nxt=None):
        chunk_step(eng, cascade, T, buf, nxt, ran, trig, out3, lookahead=not args.no_lookahead)

    eng.sync()
    torch.cuda.synchronize()
    for i in range(W):
        step(bufs[i], bufs[i + 1])
    eng.sync()
    # the cascade keeps running totals in C: nothing but the chunks in the timed loop (an older library
    # under NNSP_LIB, development A/B, has no totals: its statistics are read per step as before)
    totals = cascade and _lib.has("nnsp_cascade_totals")
    if totals:
        eng.totals_reset()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    fe_ms, nn_ms, rounds, sched, dev_ms = 0.0, 0.0, 0, 0, 0.0
    t0 = time.perf_counter()
    for i in range(K):
        step(bufs[W + i], bufs[W + i + 1])
        if cascade and not totals:
            r, f, cms = eng.last_stats()
            rounds, sched, dev_ms, fe_ms = rounds + r, sched + f, dev_ms + cms, fe_ms + eng.fe_stats()
        if not cascade:
            f, n = eng.last_timing()      # HIP events on the batch's stream around fe / proj+recur
            fe_ms += f
            nn_ms += n
    eng.sync()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if totals:   # K chunks: rounds, frames scheduled, the shared log-Mel's device ms (one launch per chunk,
        # HIP events on the cascade's stream), each chunk's device ms from its start to its rounds' end
        tot = eng.totals()
        assert tot["chunks"] == K, tot
        rounds, sched, fe_ms, dev_ms = tot["rounds"], tot["frames_run"], tot["fe_ms"], tot["chunk_ms"]
    if dist:
        dist.barrier()
    out = {"elapsed": elapsed, "frames": S * T * K, "fe_ms": fe_ms / K, "S": S}
    if cascade:
        out["rounds_per_step"] = rounds / K
        out["chunk_device_ms"] = dev_ms / K
        out["nn_frames_per_step"] = sched / K
        # one extra, untimed chunk instrumented: the nets' work serialised on
        # one stream with HIP events around each net's cold front end and NN
        # kernels of every round (the events cost a few percent, and the
        # timed steps run the nets concurrently on three streams)
        eng.set_serial(True)
        eng.set_timing(True)
        step(bufs[W + K - 1])
        eng.sync()
        eng.set_timing(False)
        eng.set_serial(False)
        out["instrumented"] = {n: dict(zip(("frames", "cold_fe_ms", "nn_ms", "rounds"), eng.net_stats(n)))
                               for n in ("vad", "kws", "s2i")}
        out["instrumented"]["shared_fe_ms"] = eng.fe_stats()
        rl, _, _ = eng.round_stats()
        out["streams_listed_per_round"] = rl.tolist()
        out["window"] = dict(zip(("next_chunk", "auto", "last_chunk_cuts"), eng.window()))
    else:
        out["nn_ms"] = nn_ms / K
    eng.close()
    return out


def roofline_blocks(args, res: dict, info: dict, profile: dict | None) -> tuple[dict, dict]:
    """The dominant kernel's roofline and the NN's (SURVEY 8(d) per-unit work)."""
    cu, clk = info["compute_units"], info["clock_khz"] * 1e3
    valu_peak = cu * 128 * clk / 1e12          # VALU lane-ops/s (4 SIMDs x 32 lanes per clock per CU)
    mul_peak, mul_src = valu_peak * 0.5, "half the VALU lane-op rate (no probe file)"
    try:   # measured v_mul_hi_i32 issue rate (profiles/microbench/valu_rates.hip), scaled to this device
        with open(os.path.join(ROOT, "profiles", "microbench", "valu_rates_mi355x.json")) as f:
            vr = json.load(f)
        mul_peak = vr["rates"]["v_mul_hi_i32"] / 1e12 * (cu * clk) / (vr["compute_units"] * vr["clock_khz"] * 1e3)
        mul_src = "measured v_mul_hi_i32 issue rate, profiles/microbench/valu_rates_mi355x.json"
    except Exception:
        pass
    issue_peak, issue_src = valu_peak / 64 / 2 * 1e12, "one wave64 VALU instruction per 2 SIMD cycles (no probe file)"
    try:   # measured v_add_u32 issue rate: the chip's VALU wave-instruction issue ceiling, scaled to this device
        issue_peak = vr["rates"]["v_add_u32"] / 64 * (cu * clk) / (vr["compute_units"] * vr["clock_khz"] * 1e3)
        issue_src = "measured v_add_u32 rate / 64 lanes (profiles/microbench/valu_rates_mi355x.json)"
    except Exception:
        pass
    mfma_peak = 5000.0                         # dense int8 MFMA Tops/s (MI355X_MICROARCH.md: 2x BF16 2.5 PF)
    cascade = args.net == "cascade"
    S, T = res["S"], args.frames
    kern = (profile or {}).get("kernels", {})
    # front end: one launch per step over all S*T frames (cascade: shared log-Mel)
    fe_ms = res["fe_ms"]
    fe_frames = S * T
    fe_ach = fe_frames * FE_MULS_PER_FRAME / (fe_ms / 1e3) / 1e12
    fe_prof = kern.get("fe_kernel[shared]" if cascade else "fe_kernel[batch]", {})
    fe_traffic = fe_prof.get("hbm_bytes_per_launch")
    fe_alg = fe_frames * fe_bytes_per_frame(cascade, T)
    fe = {"kernel": "fe_kernel", "bound": "valu", "achieved": fe_ach, "peak": mul_peak, "unit": "Tops/s",
          "frac": fe_ach / mul_peak, "traffic": fe_traffic,
          "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE, profiles/pmc_latest.json)",
          "algorithmic_bytes_per_launch": fe_alg,
          "work": "5912 integer multiplies per frame (SURVEY 8(d)) x frames per launch",
          "peak_source": mul_src, "valu_lane_peak": valu_peak, "avg_launch_ms": fe_ms,
          "frames_per_launch": fe_frames, "launches_per_step": 1,
          "hbm_achieved_GBps": fe_alg / (fe_ms / 1e3) / 1e9, "hbm_peak_GBps": 8000.0,
          # the resource that binds: VALU issue (PMC of the profiled run, profiles/pmc_latest.json)
          "valu_busy": fe_prof.get("valu_busy"),
          "valu_busy_how": "SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs), the kernel's PMC pass",
          "valu_insts_per_frame": (fe_prof["SQ_INSTS_VALU"] / fe_frames) if fe_prof.get("SQ_INSTS_VALU") else None,
          # issue-cost-weighted: the instructions' measured SIMD cycles, not one quad-cycle each
          # (profiles/fe_valu_mix.json from profiles/r05/fe_valu_mix.py: per-opcode microbench costs x the
          # frame loop's static mix -> average cycles per VALU instruction) x SQ_INSTS_VALU over the
          # launch's SIMD-cycles
          **fe_occupancy(fe_prof),
          "clock_ghz_pmc": fe_prof.get("clock_ghz")}
    # NN: MACs x 2 ops x inferences / the NN kernels' device time
    if cascade:
        ins = res["instrumented"]
        nn_ms = sum(ins[n]["nn_ms"] for n in ("vad", "kws", "s2i"))
        ops = sum(ins[n]["frames"] / 2 * NN_MACS_PER_INFERENCE[n] * 2 for n in ("vad", "kws", "s2i"))
        inf = sum(ins[n]["frames"] for n in ("vad", "kws", "s2i")) / 2
        how = ("one instrumented chunk, nets serialised on one stream, HIP events around each net's proj+recur "
               "per round; inferences = frames scheduled / 2 (speculative work past a switch included)")
        cold_ms = sum(ins[n]["cold_fe_ms"] for n in ("vad", "kws", "s2i"))
    else:
        nn_ms = res["nn_ms"]
        inf = S * T / 2
        ops = inf * NN_MACS_PER_INFERENCE[args.net] * 2
        how = "HIP events around proj+recur on the batch's stream, every timed step"
        cold_ms = 0.0
    nn_ach = ops / (nn_ms / 1e3) / 1e12 if nn_ms > 0 else 0.0
    nn_traffic = None
    nn_valu = None
    if kern:
        nn_traffic = sum(v.get("hbm_bytes_per_step", 0) for k, v in kern.items()
                         if k.startswith(("proj_kernel", "recur")))
        nn_valu = sum(v.get("valu_insts_per_step", 0) for k, v in kern.items()
                      if k.startswith(("proj_kernel", "recur"))) or None
    # the NN against VALU issue: its wave-instructions per step (PMC) over its
    # device time, against the chip's VALU issue ceiling (the MFMA line above
    # says how little of the matrix cores it uses; this one, how much of the
    # resource it is actually bound by)
    nn_issue = nn_valu / (nn_ms / 1e3) if (nn_valu and nn_ms > 0) else None
    nn = {"kernels": "proj_kernel + recur_pipe_kernel (all nets)", "bound": "mfma", "achieved": nn_ach,
          "peak": mfma_peak, "unit": "Tops/s", "frac": nn_ach / mfma_peak, "ms_per_step": nn_ms,
          "cold_fe_ms_per_step": cold_ms, "inferences_per_step": inf, "how": how,
          "work": "int8xint16 MACs per inference (VAD 14616, KWS 56448, S2I 72072) x 2 ops",
          "algorithmic_bytes_per_step": inf * NN_HBM_BYTES_PER_INFERENCE,
          "traffic_bytes_per_step": nn_traffic or None,
          "traffic_over_algorithmic": (nn_traffic / (inf * NN_HBM_BYTES_PER_INFERENCE)) if nn_traffic else None,
          "issue": {"bound": "valu", "achieved": nn_issue / 1e9 if nn_issue else None, "peak": issue_peak / 1e9,
                    "unit": "G VALU wave-instructions/s", "frac": nn_issue / issue_peak if nn_issue else None,
                    "valu_insts_per_step": nn_valu,
                    "valu_insts_per_inference": nn_valu / inf if nn_valu else None,
                    "peak_source": issue_src,
                    "how": "SQ_INSTS_VALU of proj + recur per step (PMC, profiles/pmc_latest.json) / the NN's device "
                           "time per step (ms_per_step above)"}}
    # the dominant kernel: the one with the larger device time per step
    if nn_ms > fe_ms:
        dom = {"kernel": nn["kernels"], "bound": "mfma", "achieved": nn_ach, "peak": mfma_peak, "unit": "Tops/s",
               "frac": nn["frac"], "traffic": nn_traffic, "avg_launch_ms": nn_ms, "work": nn["work"]}
        return dom, {"fe": fe, "nn": nn}
    return fe, {"nn": nn}


def fe_occupancy(fe_prof: dict) -> dict:
    try:
        with open(os.path.join(ROOT, "profiles", "fe_valu_mix.json")) as f:
            mix = json.load(f)
        avg = float(mix["avg_cycles_per_valu"])
        simd_cycles = 1024 * fe_prof["GRBM_GUI_ACTIVE"] / 8
        occ = fe_prof["SQ_INSTS_VALU"] * avg / simd_cycles
    except Exception:
        return {"valu_occupancy": None}
    return {"valu_occupancy": occ, "valu_avg_issue_cycles": avg,
            "valu_occupancy_how": "SQ_INSTS_VALU x avg SIMD cycles per VALU instruction (frame-loop opcode mix x "
                                  "microbench issue costs, profiles/fe_valu_mix.json) / (1024 SIMDs x "
                                  "GRBM_GUI_ACTIVE / 8 XCDs)"}


def load_profile(args, S: int, weights: str) -> dict | None:
    try:
        with open(args.profile_json) as f:
            pj = json.load(f)
    except Exception:
        return None
    if (pj.get("workload") == args.net and pj.get("streams") == S and pj.get("frames") == args.frames
            and pj.get("weights", "synth") == weights and pj.get("input", "noise") == args.input):
        return pj
    return None


def rank_shard(args, rank: int, world: int) -> tuple[int, int]:
    """(first global stream, streams) of this rank (nnsp_amd.shard)."""
    if args.scaling == "weak":
        per = args.streams or (32768 if args.net == "cascade" else 8192)
        return shard_streams(rank, world, per_rank=per)
    return shard_streams(rank, world, total=args.total_streams)


def spawn_ranks(n: int, argv: list[str]) -> int:
    """``bench.py --gpus N`` started as one plain process: run it again as N
    ranks under torch.distributed.run (one process per GPU, rendezvous on
    127.0.0.1) and return their exit status.  Called before this process has
    touched the GPU; the ranks inherit stdout, where rank 0 writes the one
    JSON line."""
    import socket

    with socket.socket() as s:   # a free port for the rendezvous
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + argv
    sys.stdout.flush()
    return subprocess.run(cmd).returncode


def print_rank_plan(args, rank: int, world: int, launched: bool, json_fd: int) -> None:
    """--dry-run: every rank reports its device and stream shard over a gloo
    group; rank 0 prints them as one JSON line.  Nothing touches the GPU."""
    s0, S = rank_shard(args, rank, world)
    local = int(os.environ.get("LOCAL_RANK", rank))
    me = {"rank": rank, "local_rank": local, "device": local, "first_stream": s0, "streams": S, "pid": os.getpid()}
    plan = [me]
    if launched:
        import torch.distributed as dist

        dist.init_process_group("gloo")
        plan = [None] * world
        dist.all_gather_object(plan, me)
        dist.destroy_process_group()
    if rank == 0:
        line = {"dry_run": True, "n_gpus": world, "launched_by": "torch.distributed.run" if launched
                else "plain process", "scaling": args.scaling, "net": args.net, "frames_per_step": args.frames,
                "ranks": plan}
        os.write(json_fd, (json.dumps(line) + "\n").encode())


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--net", default="cascade", choices=sorted(WORKLOADS))
    ap.add_argument("--streams", type=int, default=0,
                    help="streams per GPU (weak scaling; default 32768 for the cascade, 8192 for one net)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="strong: --total-streams split over the ranks")
    ap.add_argument("--total-streams", type=int, default=STRONG_TOTAL)
    ap.add_argument("--window", type=int, default=-1, help="cascade frames per round (-1: automatic per chunk)")
    ap.add_argument("--no-lookahead", action="store_true",
                    help="cascade: no look-ahead front end of the next chunk (overlapped with the nets)")
    ap.add_argument("--frames", type=int, default=100, help="frames per step (chunk)")
    ap.add_argument("--acc32", action="store_true")
    ap.add_argument("--build", default="shipped", choices=["shipped", "portable"],
                    help="the reference build reproduced: shipped (ARM_OPTIMIZED=1) or portable (ARM_OPTIMIZED=0, row N4)")
    ap.add_argument("--weights", default="ref", choices=["ref", "synth"])
    ap.add_argument("--input", default="mix", choices=["mix", "noise"])
    ap.add_argument("--no-stress", action="store_true",
                    help="skip the second cascade line on synthetic weights (N=1 only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # the path has no exchange step (streams are independent shards), so the
    # ranks' process group only brackets and reduces the timing: gloo, on the
    # host.  An RCCL group (nccl) measured 0.92 against 1.02 G frames/s at
    # world size 1: its streams share HIP's four hardware queues with the
    # cascade's four (GPU_MAX_HW_QUEUES=8: 0.97 G); profiles/r03/torchrun.sh
    ap.add_argument("--dist-backend", default="gloo", choices=["gloo", "nccl"],
                    help="process group of the ranks (barriers and the timing / frame-count reductions only)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--profile-json", default=os.path.join(ROOT, "profiles", "pmc_latest.json"))
    ap.add_argument("--dropin-latency", action="store_true",
                    help="time the drop-in NNSPClass_exec per frame on one stream (GPU) against the oracle on one "
                         "core; prints its own JSON line instead of the throughput line")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch the ranks and print their stream-shard plan as one JSON line; no GPU work")
    args = ap.parse_args()
    if args.dropin_latency:
        # gcc runs before this process touches the GPU (a fork/exec of a
        # process holding a HIP context is unsafe on this pool)
        lib, build = native_oracle() if not args.no_cpu_baseline else (None, None)
        import torch

        torch.cuda.set_device(0)
        res = dropin_latency(args, lib, build)
        print(json.dumps({"metric": "drop-in NNSPClass_exec latency per 10 ms frame, one stream",
                          "unit": "us/frame", "higher_is_better": False, "nets": res}))
        return

    rank, world, local, launched = dist_env()
    if launched and world != args.gpus:
        sys.exit(f"bench.py: launched with WORLD_SIZE={world} but --gpus {args.gpus}; the two must agree")
    if not launched and args.gpus > 1:
        # one process per GPU: start the ranks as children before anything here
        # touches the GPU, forward their one JSON line, exit with their status
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    # stdout carries the one JSON line and nothing else: libraries that print
    # banners there (RCCL prints its version at process-group init) write to
    # stderr instead, the line goes to the saved descriptor
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    if args.dry_run:
        print_rank_plan(args, rank, world, launched, json_fd)
        return
    # the CPU baseline runs on rank 0 at N=1 only; its pool exists before the GPU does
    pool, cpu = cpu_pool() if rank == 0 and world == 1 and not args.no_cpu_baseline else (None, None)
    import torch

    dist = None
    torch.cuda.set_device(local if launched else 0)
    if launched:   # torch.distributed.run: a process group (--dist-backend), world size 1 included
        import torch.distributed as dist

        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    from nnsp_amd import _lib
    from nnsp_amd.engine import device_info

    _lib.check(_lib.lib().nnsp_set_device(local if launched else 0), "set_device")
    s0, S = rank_shard(args, rank, world)
    res = run_workload(args, S, s0, args.weights, dist)
    elapsed, frames = reduce_run(dist, res["elapsed"], res["frames"],
                                 device="cuda" if args.dist_backend == "nccl" else "cpu")
    stress = None
    if args.net == "cascade" and world == 1 and not args.no_stress and args.weights == "ref":
        r2 = run_workload(args, S, s0, "synth")
        stress = {"weights": "synth", "value": r2["frames"] / r2["elapsed"],
                  "ms_per_step": r2["elapsed"] / args.steps * 1e3, "rounds_per_step": r2["rounds_per_step"],
                  "speculation_overhead": r2["nn_frames_per_step"] / (S * args.frames) - 1.0,
                  "shared_fe_ms": r2["fe_ms"],
                  "nn_ms": {n: r2["instrumented"][n]["nn_ms"] for n in ("vad", "kws", "s2i")}}
    if rank == 0:
        info = device_info()
        dom, extra = roofline_blocks(args, res, info,
                                     load_profile(args, S, args.weights) if args.build == "shipped" else None)
        if args.build == "portable":
            dom["note"] = ("work counted as the shipped build's 5912 multiplies per frame; the portable FFT does 16 "
                           "64-bit products per butterfly (fft.c) instead of 12 truncated ones; no PMC profile")
        value = frames / elapsed
        out = {
            "metric": "audio frames/sec (16 kHz, 10 ms hop) per node; bit-exact vs ref",
            "value": value,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "int32 (int16 PCM, q31 FFT, int8xint16 MACs)",
            "data": ("synthetic int16 PCM generated on device (SplitMix64 noise; every 4th stream replays the "
                     "reference's python/test_wavs)" if args.input == "mix" else
                     "synthetic SplitMix64 int16 PCM generated on device") +
                    ("; the reference's own def_nn*.c weights" if args.weights == "ref" else
                     "; seeded synthetic weights of the reference net shapes"),
            "config": {"workload": WORKLOADS[args.net], "net": args.net, "streams_per_gpu": S,
                       "streams_total": S * world if args.scaling == "weak" else args.total_streams,
                       "frames_per_step": args.frames, "accumulator": "32b" if args.acc32 else "64b",
                       "weights": args.weights, "input": args.input,
                       "build": "ARM_OPTIMIZED=1 (shipped)" if args.build == "shipped" else "ARM_OPTIMIZED=0 (portable)",
                       "parallelism": f"stream shards x{world}" +
                                      (f" ({'RCCL' if args.dist_backend == 'nccl' else 'gloo'} process group)" if dist else "")},
            "roofline": dom,
            **{f"roofline_{k}": v for k, v in extra.items()},
            "fe_ms_per_step": res["fe_ms"],
            "device": info,
        }
        if args.net == "cascade":
            out["cascade"] = {"rounds_per_step": res["rounds_per_step"], "window": res["window"],
                              # from the chunk's first event to its rounds' end on the device; the rest of
                              # ms_per_step is the host's turn-around between chunks (and the counter copy)
                              "chunk_device_ms": res["chunk_device_ms"],
                              "host_gap_ms": elapsed / args.steps * 1e3 - res["chunk_device_ms"],
                              "lookahead_front_end": not args.no_lookahead,
                              "speculation_overhead": res["nn_frames_per_step"] / (S * args.frames) - 1.0,
                              "instrumented_chunk": res["instrumented"],
                              "streams_listed_per_round": res["streams_listed_per_round"]}
            if stress:
                out["cascade_synthetic_weights"] = stress
        else:
            out["nn_ms_per_step"] = res["nn_ms"]
        if pool is not None:
            with pool:
                out["cpu_baseline"] = cpu_baseline(pool, cpu, args.net, args.acc32, args.weights,
                                                   args.input == "mix", args.cpu_seconds,
                                                   portable=args.build == "portable")
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
