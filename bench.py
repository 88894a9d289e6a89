#!/usr/bin/env python3
"""Benchmark: ICP iterations/s (cfg1, cfg3) + RANSAC hypotheses/s (cfg2) on synthetic pairs.

BASELINE.json metric "ICP iterations/sec + RANSAC hypotheses/sec, 100k↔100k pts, 1/2/4/8 GPU".

* step (the timed unit of the headline) = one full cfg1 ICP run: 100k source ↔ 100k target
  points per GPU, 50 point-to-plane iterations (convergence disabled → exactly 50 updates, 51 NN
  evaluations), brute-force radius-bounded NN (r = 0.4·0.3), exact fp64 correspondences
  (nnkey.h), fp64 terms/solve, all device resident.  value = ICP iterations/s summed over ranks;
  N > 1 is weak scaling (one cfg1 block per GPU): the north-star's rule shards the TARGET only
  when the cloud would not fit one GPU's HBM (M3D_TARGET_SHARD_BYTES), else the sources
  (`--shard target|source` forces either).  The collectives run inside libm3d over RCCL
  (m3d_comm_*, `"comm": "libm3d-rccl"`); torch.distributed only carries the RCCL unique id.
* "cfg3": BASELINE cfg3 — the 1M ↔ 1M pair, target sharded over the N GPUs (1M/N targets per
  rank, one shared fp32 frame, sources replicated), MIN of the fp64 NN keys + MIN of the
  claims + SUM of the 32 terms per iteration: STRONG scaling of one fixed problem, value = ICP
  iterations/s of that problem.  Brute-force NN (north_star) and, beside it, the uniform grid.
  `--config cfg3` makes it the headline line.
* "ransac": cfg2 — benchmark_ransac.py's loop (a1 sample + Kabsch, a2 ‖d‖ < 1.5·v scoring) at
  Nc = 1e5, H = 1e5 hypotheses per GPU, counter sampler seed 42, no early stop; N > 1 shards the
  hypothesis ids and all-reduces MAX of the packed (count, ~id) key (m3d_ransac_best_allreduce).
* "ransac_api": the reference harness's own calling pattern through the drop-in
  (matcher.ransac.compute_step_transformation + evaluate_inlier_ratio per hypothesis,
  benchmark_ransac.py:87-125) at Nc = 5k and 1e5: ms per call next to BASELINE.md's numbers.
* roofline (every section): the kernel's ALGORITHMIC work ÷ its average launch time, measured
  with HIP events recorded by the library on the launch stream around every launch (a second
  timed pass of the same steps; `value` comes from the pass without events), ÷ the peak of the
  pipe the kernel runs on.  The NN screen and the RANSAC residuals run on the FP16 matrix pipe
  (DESIGN.md §3.2a/§3.5 — a deviation from north_star's "MFMA not used" that beats the FP32
  vector roof), so `frac` = SURVEY §8(d)'s 8 flop per (source, target) pair resp. 27 flop per
  (hypothesis, correspondence) pair ÷ the dense FP16 MFMA peak (2.5 PFLOP/s); `mfma_issue_frac`
  gives the issued fp16 MACs (32 resp. 96 flop per pair) against the same peak.  The grid NN is
  priced in GB/s on 28·Ns + 16·Nt algorithmic bytes per launch.  traffic = HBM bytes per launch
  from the committed rocprofv3 PMC summary (profiles/pmc_*.json), or null.
* cpu_baseline (rank 0, N = 1): the oracle restatement (scipy cKDTree + numpy point-to-plane;
  numpy a1+a2) timed on the host cores this process may use (affinity ∩ cgroup quota).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "3d-matching_amd"))

VALU_FP32_PEAK_TF = 157.3   # MI355X_MICROARCH.md: Peak FP32 (vector)
HBM_PEAK_GBS = 8000.0
MFMA_F16_PEAK_TF = 2500.0   # MI355X_MICROARCH.md: Peak BF16/FP16 MFMA, dense
NN_FLOP_PER_PAIR = 8        # 3 sub + 1 mul + 2 FMA: the algorithmic basis
NN_MFMA_FLOP_PER_PAIR = 32  # 16 fp16 MACs per (target, query) pair in v_mfma_f32_32x32x16_f16
SCORE_FLOP_PER_PAIR = 27    # 9 FMA transform + 3 sub + (1 mul + 2 FMA) + 1 cmp
SCORE_MFMA_FLOP_PER_PAIR = 96  # 3 x v_mfma_f32_32x32x16_f16 (16 fp16 MACs each) per pair
NN_NOTE = ("north_star expected VALU; the |t|^2-2q.t screen runs on the FP16 matrix pipe "
           "(DESIGN.md 3.5): frac = the 8-flop/pair algorithmic rate / the dense FP16 MFMA peak of that pipe")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=["cfg1", "cfg3"], default="cfg1",
                    help="headline: cfg1 (100k<->100k per GPU, weak) or cfg3 (1M<->1M, strong)")
    ap.add_argument("--ns", type=int, default=100_000)
    ap.add_argument("--nt", type=int, default=100_000, help="target points per GPU (cfg1)")
    ap.add_argument("--icp-iters", type=int, default=50)
    ap.add_argument("--cfg3-n", type=int, default=1_000_000)
    ap.add_argument("--cfg3-iters", type=int, default=50)  # as cfg1: the unseeded first evaluation amortised alike
    ap.add_argument("--cfg3-steps", type=int, default=2)
    ap.add_argument("--no-cfg3", action="store_true")
    ap.add_argument("--nc", type=int, default=100_000)
    ap.add_argument("--hyps", type=int, default=100_000, help="RANSAC hypotheses per GPU per run")
    ap.add_argument("--ransac-steps", type=int, default=20,
                    help="timed RANSAC runs (~1.5 ms each): enough that the sync at either end "
                         "of the timed region does not weigh on the per-run time")
    ap.add_argument("--no-ransac", action="store_true")
    ap.add_argument("--ransac-warmup-s", type=float, default=0.5,
                    help="untimed RANSAC runs for at least this long before the timed ones")
    ap.add_argument("--no-ransac-api", action="store_true")
    ap.add_argument("--no-grid", action="store_true")
    ap.add_argument("--no-cfg4", action="store_true")
    ap.add_argument("--cfg4-mesh", type=int, default=300,
                    help="cfg4 source mesh rings (segments = 2x; target mesh 10%% finer)")
    ap.add_argument("--shard", choices=["auto", "target", "source"], default="auto",
                    help="N>1 cfg1 sharding: target (MIN of the NN keys + claims, SUM of the terms), "
                         "source (target replicated, SUM of the terms only), or auto: the "
                         "north-star's rule -- shard the target only when it would not fit one "
                         "GPU's HBM budget (M3D_TARGET_SHARD_BYTES, default 64 GiB), else source")
    ap.add_argument("--target-shards", choices=["spatial", "index"], default="spatial",
                    help="target shards of the target-sharded runs (cfg3, and cfg1 under --shard "
                         "target): spatial = slabs of the longest axis (m3d.dist.spatial_shards; "
                         "a query whose box misses a rank's slab leaves its scan at once), index = "
                         "ranges of the unordered cloud (every shard spans the whole surface)")
    ap.add_argument("--comm", choices=["lib", "torch"], default="lib",
                    help="N>1 collectives: libm3d's RCCL communicator, or torch.distributed")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=8.0, help="seconds per CPU baseline leg")
    ap.add_argument("--launch-check", action="store_true",
                    help="bring up the ranks and the process group only, print the line with the "
                         "rank count and exit (no GPU work: the launcher's CPU test)")
    return ap.parse_args()


def visible_gpu_count() -> int:
    """GPUs this job may use, counted in a throwaway child so that the launcher itself never
    initialises the GPU (it starts the ranks afterwards)."""
    import subprocess

    try:
        out = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                             capture_output=True, text=True, timeout=600)
        return int(out.stdout.strip().splitlines()[-1])
    except Exception as e:  # reported: the caller refuses to launch
        print(f"[bench] could not count GPUs: {e}", file=sys.stderr)
        return 0


def launch_ranks(args) -> int:
    """`bench.py --gpus N` (N > 1) without WORLD_SIZE: start N ranks, one per GPU, under
    torch.distributed.run as a CHILD process (this process has not touched the GPU and never
    execs), and return its exit code.  Refuses, without printing a line, when fewer than N GPUs
    are visible — an N = 1 line for --gpus N is never printed.  M3D_BENCH_SAME_DEVICE=1 (every
    rank on cuda:0, the functional rehearsal) skips the count."""
    import socket
    import subprocess

    n = args.gpus
    if os.environ.get("M3D_BENCH_SAME_DEVICE") != "1":
        have = visible_gpu_count()
        if have < n:
            print(f"[bench] --gpus {n} needs {n} visible GPUs, this job sees {have}: refusing "
                  "(one rank per GPU; RCCL cannot place two ranks on one device)", file=sys.stderr)
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", str(ROOT / "bench.py"), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    return subprocess.call(cmd, env=env)


def _g(d, *path):
    """d[path[0]][path[1]]..., None where any level is missing."""
    for k in path:
        if not isinstance(d, dict) or d.get(k) is None:
            return None
        d = d[k]
    return d


def _r(x, nd=4):
    return None if x is None else (round(x, nd) if isinstance(x, float) else x)


# the fields of `summary`: the sub-legs the driver's truncated stdout tail must
# still show — the LAST key of the JSON line, kept under ~600 characters
SUMMARY_FIELDS = ("icp_brute", "icp_brute_frac", "icp_grid", "icp_grid_frac", "cfg1_cold_grid_ms",
                  "cfg1_strong", "cfg1_strong_grid", "ransac", "ransac_frac", "ransac_strong",
                  "ransac_nc3e5", "cfg3_brute", "cfg3_grid", "n_gpus", "comm_ranks")


def build_summary(line: dict) -> dict:
    """The compact digest of a bench line (every SUMMARY_FIELDS key; None where a leg did not run):
    ICP it/s brute + grid with their roofline fractions, the cold cfg1 grid stages (clouds / loop
    / iterations / total ms), the strong-scaling legs, RANSAC hyp/s (cfg2, its strong split, the
    Nc = 3e5 secondary), cfg3 brute + grid it/s, n_gpus and the communicator's rank count."""
    cold = _g(line, "cfg1_cold", "grid")
    out = {
        "icp_brute": _r(line.get("value"), 1), "icp_brute_frac": _r(_g(line, "roofline", "frac")),
        "icp_grid": _r(_g(line, "icp_grid", "value"), 1),
        "icp_grid_frac": _r(_g(line, "icp_grid", "roofline", "frac")),
        "cfg1_cold_grid_ms": (None if cold is None else
                              [_r(cold.get(k), 3) for k in ("clouds_ms", "loop_create_ms", "iterations_ms", "total_ms")]),
        "cfg1_strong": _r(_g(line, "cfg1_strong", "value"), 1),
        "cfg1_strong_grid": _r(_g(line, "cfg1_strong", "grid_value"), 1),
        "ransac": _r(_g(line, "ransac", "value"), 0), "ransac_frac": _r(_g(line, "ransac", "roofline", "frac")),
        "ransac_strong": _r(_g(line, "ransac", "strong", "value"), 0),
        "ransac_nc3e5": _r(_g(line, "ransac", "nc3e5", "value"), 0),
        "cfg3_brute": _r(_g(line, "cfg3", "value"), 2), "cfg3_grid": _r(_g(line, "cfg3", "grid", "value"), 1),
        "n_gpus": line.get("n_gpus"), "comm_ranks": _g(line, "config", "comm_ranks"),
    }
    assert tuple(out) == SUMMARY_FIELDS
    return out


def launch_check(args, world, rank):
    """--launch-check: the process group over gloo (no GPU), a SUM of ones to count the ranks
    that actually joined, and rank 0's line."""
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
        one = torch.ones(1, dtype=torch.int64)
        dist.all_reduce(one)
        joined, pg_world = int(one.item()), dist.get_world_size()
    else:
        joined, pg_world = 1, 1
    if pg_world != args.gpus or joined != args.gpus:
        print(f"[bench] rank {rank}: process group has {pg_world} ranks ({joined} joined), --gpus {args.gpus}",
              file=sys.stderr)
        return 3
    if rank == 0:
        line = {"metric": "launch check", "value": None, "n_gpus": pg_world, "ranks_joined": joined,
                "launch_check": True, "config": {"comm": "gloo", "comm_ranks": joined}}
        line["summary"] = build_summary(line)  # the same last key as a measured line
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def pmc_traffic(kernel_substr: str, shape: str = ""):
    """HBM bytes per launch from the newest committed PMC summary (profiles/pmc_rNN.json at the
    bench's cfg1 / cfg2 shapes; shape="1m": profiles/pmc_rNN_1m.json, the 1M x 1M grid)."""
    import re

    pat = re.compile(r"pmc_r\d+" + (f"_{shape}" if shape else "") + r"\.json$")
    files = sorted(f for f in (ROOT / "profiles").glob("pmc_*.json") if pat.search(f.name))
    for f in reversed(files):
        try:
            d = json.loads(f.read_text())
        except Exception:
            continue
        for k, v in d.get("kernels", {}).items():
            if kernel_substr in k and v.get("hbm_bytes_per_launch") is not None:
                return float(v["hbm_bytes_per_launch"]), f.name
    return None, None


def host_cores():
    """CPU threads this process may use: sched affinity ∩ the cgroup CPU quota."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(p)))
    except Exception:
        pass
    used = min(aff, quota) if quota else aff
    env = {k: os.environ.get(k) for k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS")}
    return used, {"affinity": aff, "cgroup_quota": quota, **env}


def nn_roofline(ns, nt, avg_ms, launches, terms_ms):
    algo = NN_FLOP_PER_PAIR * ns * nt / (avg_ms * 1e-3) / 1e12
    issued = NN_MFMA_FLOP_PER_PAIR * ns * nt / (avg_ms * 1e-3) / 1e12
    traffic, src = pmc_traffic("nn_mfma_kernel")
    return {"bound": "mfma", "kernel": "nn_mfma_kernel", "achieved": algo, "peak": MFMA_F16_PEAK_TF,
            "unit": "TFLOP/s", "frac": algo / MFMA_F16_PEAK_TF, "traffic": traffic,
            "traffic_source": src, "avg_launch_ms": avg_ms, "launches": launches,
            "flop_per_pair": NN_FLOP_PER_PAIR, "pairs_per_launch": ns * nt,
            "mfma_issued_tflops": issued, "mfma_issue_frac": issued / MFMA_F16_PEAK_TF,
            "vs_fp32_valu_roof": algo / VALU_FP32_PEAK_TF, "terms_avg_launch_ms": terms_ms,
            "note": NN_NOTE}


def main():
    args = parse()
    if args.gpus < 1:
        print("[bench] --gpus must be >= 1", file=sys.stderr)
        sys.exit(2)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))  # before anything here touches the GPU
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"[bench] WORLD_SIZE={world} but --gpus {args.gpus}: refusing to print a mislabelled line",
              file=sys.stderr)
        sys.exit(2)
    if args.launch_check:
        sys.exit(launch_check(args, world, rank))

    import numpy as np
    import torch
    import torch.distributed as dist

    # M3D_BENCH_DIST=1 (under torch.distributed.run): take the N > 1 code path even at world 1 —
    # the nccl process group, the libm3d RCCL communicator beside it and the sharded protocols —
    # a rehearsal of the driver's multi-GPU runs on a one-GPU box (tools/gpu_dist1_rehearsal.sh)
    multi = world > 1 or os.environ.get("M3D_BENCH_DIST") == "1"
    if multi:
        # M3D_BENCH_SAME_DEVICE=1 + M3D_BENCH_BACKEND=gloo: every rank on cuda:0 over gloo — a
        # functional rehearsal of the N > 1 path on a one-GPU box (RCCL refuses two ranks on one
        # GPU, so that rehearsal uses --comm torch); the real runs are one rank per GPU
        same = os.environ.get("M3D_BENCH_SAME_DEVICE") == "1"
        backend = os.environ.get("M3D_BENCH_BACKEND", "nccl")
        torch.cuda.set_device(0 if same else local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", 0 if same else local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from m3d import _lib, synth
    from m3d import dist as D
    from m3d.core import RESULT_WORDS, Cloud, CorrSet, IcpLoop, RansacOutcome, RansacParams, context

    ctx = context()
    comm, comm_name = None, "none"
    if multi:
        if args.comm == "lib":
            try:
                from m3d.comm import LibComm

                comm, comm_name = LibComm(rank, world), "libm3d-rccl"
            except Exception as e:  # reported, never silent
                print(f"[bench] libm3d RCCL communicator unavailable ({e}); using torch.distributed",
                      file=sys.stderr)
        if comm is None:
            comm, comm_name = D.TorchComm(), f"torch.distributed-{dist.get_backend()}"
    # the rank count the line reports is the one the collectives actually reach: a SUM of ones
    # through the same communicator the hot path uses (RCCL inside libm3d, or torch.distributed)
    comm_ranks = 1
    if multi:
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"[bench] process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
        one = torch.ones(1, dtype=torch.int64, device=dev)
        comm.sum_(one)
        torch.cuda.synchronize()
        comm_ranks = int(one.item())
        if comm_ranks != world:
            raise SystemExit(f"[bench] {comm_name} reached {comm_ranks} ranks, world {world}")

    def barrier():
        if multi:
            dist.barrier()
            torch.cuda.synchronize()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def timed(fn, steps, kernels):
        """(elapsed s of `steps` × fn without events, elapsed with events, {kernel: (ms, n)})."""
        out = []
        prof = {}
        for events in (False, True):
            ctx.profile(events)
            for k in kernels:
                ctx.profile_read(k)
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                fn()
            torch.cuda.synchronize()
            barrier()
            out.append(max_over_ranks(time.perf_counter() - t0))
            if events:
                prof = {k: ctx.profile_read(k) for k in kernels}
            ctx.profile(False)
        return out[0], out[1], prof

    # ------------------------------------------------------------------ ICP loop runner
    def icp_runner(loop, iters, mode, off=0, ns_total=0):
        """One ICP run of `iters` updates (iters + 1 evaluations) on this rank."""
        drv = None
        if mode == "source" and comm_name != "libm3d-rccl":
            drv = D.SourceShardedIcp(loop, loop.src.n, ns_total, dev, comm=comm)
        elif mode == "target" and comm_name != "libm3d-rccl":
            drv = D.ShardedIcp(loop, off, loop.src.n, dev, comm=comm)
        if mode == "single":  # setup beside the loop object: the steps' HIP graph, captured once
            loop.reset(np.eye(4))
            loop.prepare_steps(iters + 1)

        def run():
            loop.reset(np.eye(4))
            if mode == "single":
                loop.steps(iters + 1)  # the library enqueues the iterations natively
            elif drv is None:  # libm3d issues the RCCL collectives between its own kernels
                if mode == "source":
                    loop.source_shard_steps(comm, iters + 1)
                else:
                    loop.shard_steps(comm, off, iters + 1)
            else:
                for _ in range(iters + 1):
                    drv.iteration()
        return run

    # ------------------------------------------------------------------ cfg1: ICP
    ns, nt, iters = args.ns, args.nt, args.icp_iters
    r = 0.4 * 0.3
    shard = args.shard
    if shard == "auto":
        # north_star: "shards the target cloud ... with an RCCL all-reduce of per-shard
        # (min_dist, argmin) ... only for clouds large enough to saturate one GPU's HBM"; a
        # replicated cloud costs 64 B per point
        budget = float(os.environ.get("M3D_TARGET_SHARD_BYTES", 64 * 2**30))
        shard = "target" if 64.0 * nt * world > budget else "source"
    mode1 = "single" if not multi else shard
    if mode1 == "source":  # weak scaling: ns sources per rank against the whole (replicated) target
        src_all, tgt_all, nrm_all, T_true = synth.icp_pair(ns * world, nt, seed=0)
        src = src_all[rank * ns:(rank + 1) * ns]
        off = 0
        tgt_c = Cloud(tgt_all, nrm_all)
    else:  # single device, or target-sharded: nt targets per rank, sources replicated
        src, tgt_all, nrm_all, T_true = synth.icp_pair(ns, nt * world, seed=0)
        off = rank * nt
        if not multi:
            tgt_c = Cloud(tgt_all, nrm_all)
        else:  # the target as the shards see it: spatially ordered slabs (or index ranges)
            c_all = tgt_all.mean(axis=0)
            if args.target_shards == "spatial":
                perm1, b1 = D.spatial_shards(tgt_all, world)
                tgt_all, nrm_all = tgt_all[perm1], nrm_all[perm1]
                off, nt_r = int(b1[rank]), int(b1[rank + 1] - b1[rank])
            else:
                nt_r = nt
            tgt_c = Cloud(tgt_all[off:off + nt_r], nrm_all[off:off + nt_r], center=c_all)
    src_c = Cloud(src)
    K_NN, K_TERMS, K_COMM = _lib.KERNEL_NN, _lib.KERNEL_TERMS, _lib.KERNEL_COMM

    def split_times(prof, el_ev, evals):
        """Per evaluation (one NN + terms + exchange), from the events pass: the NN, terms and
        RCCL all-reduce times on their own streams (the split target-shard exchange runs half of
        its keys beside the NN, so the three need not add up to the iteration), max over ranks."""
        def per(k):
            return None if k not in prof or prof[k][1] == 0 else max_over_ranks(prof[k][0] / evals)
        return {"per_evaluation_ms_with_events": max_over_ranks(el_ev) / evals * 1e3,
                "nn_ms_per_evaluation": per(K_NN), "terms_ms_per_evaluation": per(K_TERMS),
                "exchange_ms_per_evaluation": per(K_COMM),
                "allreduces_per_evaluation": None if K_COMM not in prof else prof[K_COMM][1] / evals,
                "exchange_note": ("library RCCL all-reduces timed by events on their streams"
                                  if comm_name == "libm3d-rccl" else "exchange not issued by the library")}

    def bench_icp(nn):
        loop = IcpLoop(src_c, tgt_c, r, relative_fitness=-1.0, relative_rmse=-1.0, max_iteration=iters, nn=nn)
        if mode1 == "source":
            loop.set_source_total(ns * world)
        run = icp_runner(loop, iters, mode1, off, ns * world)
        for _ in range(args.warmup):
            run()
        torch.cuda.synchronize()
        el, el_ev, prof = timed(run, args.steps, (K_NN, K_TERMS))
        (nn_ms, nn_n), (t_ms, t_n) = prof[K_NN], prof[K_TERMS]
        return el, el_ev, max_over_ranks(nn_ms / max(nn_n, 1)), nn_n, t_ms / max(t_n, 1), loop.result()

    el, el_ev, nn_avg_ms, nn_n, terms_avg_ms, res = bench_icp("brute")
    icp_value = world * iters * args.steps / el
    err = float(np.abs(res.transformation - T_true).max())
    cfg1 = {
        "value": icp_value, "ms_per_step": el / args.steps * 1e3,
        "ms_per_step_with_kernel_events": el_ev / args.steps * 1e3,
        "workload": (f"cfg1: {ns}<->{nt} synthetic pair per GPU, {iters} point-to-plane ICP "
                     f"iterations, brute-force NN (r={r:g}), "
                     + ("1 GPU" if not multi else
                        (f"sources sharded over {world} GPUs ({ns} per GPU), target replicated (SUM terms)"
                         if mode1 == "source" else
                         f"target sharded over {world} GPUs ({nt} per GPU), sources replicated "
                         "(MIN keys + MIN claims + SUM terms)"))),
        "roofline": nn_roofline(ns, nt, nn_avg_ms, nn_n, terms_avg_ms),
        "check": {"icp_fitness": res.fitness, "icp_rmse": res.inlier_rmse, "max_abs_err_vs_T_true": err},
    }

    icp_grid = None
    if not args.no_grid:
        tg0 = time.perf_counter()
        IcpLoop(src_c, tgt_c, r, max_iteration=0, nn="grid")  # builds both clouds' grids once
        torch.cuda.synchronize()
        build_ms = (time.perf_counter() - tg0) * 1e3
        gel, gel_ev, g_ms, g_n, g_terms_ms, gres = bench_icp("grid")
        g_bytes = 28 * ns + 16 * nt
        g_gbs = g_bytes / (g_ms * 1e-3) / 1e9
        icp_grid = {
            "metric": "ICP iterations/sec (cfg1 workload, uniform-grid radius NN)",
            "value": world * iters * args.steps / gel, "unit": "ICP iter/s (100k src x 100k tgt per GPU)",
            "ms_per_step": gel / args.steps * 1e3, "grid_build_ms": build_ms,
            "ms_per_step_with_kernel_events": gel_ev / args.steps * 1e3,
            "same_result_as_brute": bool(np.array_equal(gres.transformation, res.transformation)),
            "roofline": {"bound": "hbm", "kernel": "grid_nn_batched_kernel", "achieved": g_gbs,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": g_gbs / HBM_PEAK_GBS,
                         "traffic": pmc_traffic("grid_nn")[0], "avg_launch_ms": g_ms,
                         "launches": g_n, "bytes_per_launch": g_bytes,
                         "terms_avg_launch_ms": g_terms_ms,
                         "note": "priced against HBM, but not HBM-bound: one resident round of "
                                 "gather waves (~6 us each), the vector-memory data-return path "
                                 "~70% busy (TD_TD_BUSY; DESIGN.md 3.8, profiles/r05_grid_scan)"},
        }

    # ------------------------------------------------------------------ cfg1 strong scaling
    # BASELINE metric as worded ("100k<->100k pts, 1/2/4/8 GPU"): the FIXED cfg1 pair over the N
    # GPUs — sources sharded ns/N per rank against the replicated target, SUM of the 32 term slots
    # (SURVEY §8(e) "ICP alternative"), value = ICP iterations/s of that one problem.  N = 1: the
    # headline run itself (the same workload), so SCALE's N = 1 line equals BENCH.
    cfg1_strong = None
    if not multi:
        cfg1_strong = {"value": cfg1["value"], "ms_per_step": cfg1["ms_per_step"],
                       "grid_value": None if icp_grid is None else icp_grid["value"],
                       "note": "N = 1: the headline cfg1 run (same workload)"}
    else:
        s1, t1, n1, T1 = synth.icp_pair(ns, nt, seed=0)  # the N = 1 pair
        o1, c1 = D.shard_bounds(ns, world, rank)
        s1c, t1c = Cloud(s1[o1:o1 + c1]), Cloud(t1, n1)
        cfg1_strong = {"workload": f"cfg1 fixed pair: {ns}<->{nt}, {iters} iterations, sources sharded "
                                   f"over {world} GPUs ({c1} on rank {rank}), target replicated, SUM terms",
                       "scaling": "strong", "unit": "ICP iter/s (one 100k x 100k problem)"}
        for nn in ("brute",) + (() if args.no_grid else ("grid",)):
            lp = IcpLoop(s1c, t1c, r, relative_fitness=-1.0, relative_rmse=-1.0, max_iteration=iters, nn=nn)
            lp.set_source_total(ns)
            run = icp_runner(lp, iters, "source", 0, ns)
            for _ in range(args.warmup):
                run()
            torch.cuda.synchronize()
            e1, e1_ev, prof = timed(run, args.steps, (K_NN, K_TERMS, K_COMM))
            rs1 = lp.result()
            sec = {"value": iters * args.steps / e1, "ms_per_step": e1 / args.steps * 1e3,
                   "nn_avg_launch_ms": max_over_ranks(prof[K_NN][0] / max(prof[K_NN][1], 1)),
                   "fitness": rs1.fitness, "max_abs_err_vs_T_true": float(np.abs(rs1.transformation - T1).max())}
            sec.update(split_times(prof, e1_ev, args.steps * (iters + 1)))
            if nn == "brute":
                cfg1_strong.update(sec)
            else:
                cfg1_strong["grid_value"] = sec["value"]
                cfg1_strong["grid"] = sec
            del lp
        del s1c, t1c

    # ------------------------------------------------------------------ cfg1 cold call
    # What the reference pays per refine_registration call (icp.py:42-48 builds its KD-tree every
    # call): fresh device clouds (H2D + centring + fp32 packing), the loop object (grids, Morton
    # source copy, fp16 MFMA tiles, target records) and the 50 iterations, per stage (synchronised
    # between stages); plus the drop-in refine_registration on fresh Ply-likes (grid NN, Open3D's
    # default convergence criteria).
    cfg1_cold = None
    if rank == 0 and world == 1:
        cfg1_cold = bench_cold(args, src, tgt_all[:nt], nrm_all[:nt], r, iters, reps=7)

    # ------------------------------------------------------------------ cfg3: 1M <-> 1M, strong
    cfg3 = None
    if not args.no_cfg3 or args.config == "cfg3":
        n3, it3 = args.cfg3_n, args.cfg3_iters
        s3, t3, nr3, T3 = synth.icp_pair(n3, n3, seed=0)
        o3, c3 = D.shard_bounds(n3, world, rank)
        s3c = Cloud(s3)
        shards3 = "none"
        if not multi:
            t3c = Cloud(t3, nr3)
        else:
            c3_all = t3.mean(axis=0)
            t3s, nr3s = t3, nr3
            if args.target_shards == "spatial":  # slabs: a query whose box misses a slab leaves at once
                perm3, b3 = D.spatial_shards(t3, world)
                t3s, nr3s = t3[perm3], nr3[perm3]
                o3, c3 = int(b3[rank]), int(b3[rank + 1] - b3[rank])
            shards3 = args.target_shards
            t3c = Cloud(t3s[o3:o3 + c3], nr3s[o3:o3 + c3], center=c3_all)
            del t3s, nr3s
        mode3 = "single" if not multi else "target"
        cfg3 = {"metric": "ICP iterations/sec (cfg3: 1M<->1M pair, target sharded over the GPUs, strong scaling)",
                "unit": "ICP iter/s (whole 1M x 1M problem)", "scaling": "strong",
                "workload": f"cfg3: {n3}<->{n3} synthetic pair, {it3} point-to-plane iterations per step, "
                            f"target sharded over {world} GPU(s) ({shards3} shards, {c3} targets on rank "
                            f"{rank}), sources replicated, MIN fp64 keys + MIN claims + SUM terms per iteration",
                "target_shards": shards3,
                "steps": args.cfg3_steps, "icp_iterations_per_step": it3}
        for nn in ("brute", "grid"):
            lp = IcpLoop(s3c, t3c, r, relative_fitness=-1.0, relative_rmse=-1.0, max_iteration=it3, nn=nn)
            run = icp_runner(lp, it3, mode3, o3)
            run()
            torch.cuda.synchronize()
            e3, e3_ev, prof = timed(run, args.cfg3_steps, (K_NN, K_TERMS, K_COMM))
            (m, n), (tm, tn) = prof[K_NN], prof[K_TERMS]
            avg = max_over_ranks(m / max(n, 1))
            r3 = lp.result()
            sec = {"value": it3 * args.cfg3_steps / e3, "ms_per_iteration": e3 / (it3 * args.cfg3_steps) * 1e3,
                   "ms_per_iteration_with_kernel_events": e3_ev / (it3 * args.cfg3_steps) * 1e3,
                   "nn_avg_launch_ms": avg, "terms_avg_launch_ms": tm / max(tn, 1),
                   "fitness": r3.fitness, "max_abs_err_vs_T_true": float(np.abs(r3.transformation - T3).max())}
            if multi:
                sec.update(split_times(prof, e3_ev, args.cfg3_steps * (it3 + 1)))
                # the same loop with the keys exchanged in one piece (no overlap with the NN)
                del lp
                lp = IcpLoop(s3c, t3c, r, relative_fitness=-1.0, relative_rmse=-1.0, max_iteration=it3, nn=nn,
                             split=False)
                run = icp_runner(lp, it3, mode3, o3)
                run()
                torch.cuda.synchronize()
                e3n, e3n_ev, profn = timed(run, args.cfg3_steps, (K_NN, K_TERMS, K_COMM))
                sec["split_off"] = {"value": it3 * args.cfg3_steps / e3n,
                                    "ms_per_iteration": e3n / (it3 * args.cfg3_steps) * 1e3,
                                    "same_result": bool(np.array_equal(lp.result().transformation, r3.transformation)),
                                    **split_times(profn, e3n_ev, args.cfg3_steps * (it3 + 1))}
            if nn == "brute":
                sec["roofline"] = nn_roofline(n3, c3, avg, n, tm / max(tn, 1))
                sec["roofline"]["note"] = "per rank: " + NN_NOTE
                cfg3.update(sec)
            else:
                g_bytes = 28 * n3 + 16 * c3
                sec["roofline"] = {"bound": "hbm", "kernel": "grid_nn_batched_kernel",
                                   "achieved": g_bytes / (avg * 1e-3) / 1e9, "peak": HBM_PEAK_GBS,
                                   "unit": "GB/s", "frac": g_bytes / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                   "bytes_per_launch": g_bytes,
                                   "traffic": pmc_traffic("grid_nn", "1m")[0] if world == 1 else None}
                cfg3["grid"] = sec
            del lp
        del s3c, t3c
        # the same pair from nothing (H2D + centring, grids, Morton copy, records; the 1M cold
        # path of refine_registration, which Open3D pays per call with its KD-tree build)
        if rank == 0 and world == 1:
            cfg3["cold"] = bench_cold(args, s3, t3, nr3, r, it3, reps=2, nns=("grid",), tag="cfg3")

    # ------------------------------------------------------------------ cfg2: RANSAC
    ransac = None
    if not args.no_ransac:
        nc, H = args.nc, args.hyps
        rs_src, rs_tgt, corr, _ = synth.ransac_pair(nc, seed=42)
        cs = CorrSet(rs_src, rs_tgt, corr)
        thr = 0.3 * 1.5
        params = RansacParams(max_iter=H, seed=42, thr=thr, mode=_lib.SCORE_NORM, early_stop=False,
                              hyp0=rank * H)
        res_buf = torch.zeros(RESULT_WORDS, dtype=torch.int64, device=dev)
        key = torch.zeros(1, dtype=torch.int64, device=dev)

        def ransac_run():
            # enqueued without a host round trip (m3d_ransac_run_async): runs go back to back
            cs.run_async(params, res_buf)
            if multi:  # best over ranks: highest count, lowest global id (device-side key)
                if comm_name == "libm3d-rccl":
                    cs.best_allreduce(comm, res_buf, rank * H, key)
                else:
                    key.copy_(res_buf[19:20] * (1 << 32) + (0xFFFFFFFF - (rank * H + res_buf[17:18])))
                    comm.max_(key)

        # warm-up: the clocks drop while the host prepares the RANSAC data with the GPU idle, so
        # run about --ransac-warmup-s seconds of untimed runs (the same count on every rank: the
        # runs of N > 1 contain a collective)
        ransac_run()
        torch.cuda.synchronize()
        t_w = time.perf_counter()
        ransac_run()
        torch.cuda.synchronize()
        t_one = max_over_ranks(time.perf_counter() - t_w)
        for _ in range(max(0, int(args.ransac_warmup_s / max(t_one, 1e-6)) - 2)):
            ransac_run()
        torch.cuda.synchronize()
        K_SC, K_KB = _lib.KERNEL_SCORE, _lib.KERNEL_KABSCH
        rel, rel_ev, prof = timed(ransac_run, args.ransac_steps, (K_SC, K_KB))
        out = RansacOutcome.from_device(res_buf, nc)
        (sc_ms, sc_n), (kb_ms, kb_n) = prof[K_SC], prof[K_KB]
        sc_avg = max_over_ranks(sc_ms / max(sc_n, 1))
        hyps_per_launch = H / max(sc_n // args.ransac_steps, 1)
        pairs = nc * hyps_per_launch
        sc_algo = SCORE_FLOP_PER_PAIR * pairs / (sc_avg * 1e-3) / 1e12
        sc_issued = SCORE_MFMA_FLOP_PER_PAIR * pairs / (sc_avg * 1e-3) / 1e12
        # the FIXED H = 1e5 batch split over the ranks (hypothesis ids [off, off + cnt) per rank,
        # MAX of the packed key): strong scaling of one cfg2 run; N = 1: the run above
        ransac_strong = {"value": world * H * args.ransac_steps / rel, "ms_per_run": rel / args.ransac_steps * 1e3,
                         "hyps_per_run": H, "note": "N = 1: the cfg2 run above (same workload)"}
        if multi:
            o2, c2 = D.shard_bounds(H, world, rank)
            p2 = RansacParams(max_iter=c2, seed=42, thr=thr, mode=_lib.SCORE_NORM, early_stop=False, hyp0=o2)

            def ransac_strong_run():
                cs.run_async(p2, res_buf)
                if comm_name == "libm3d-rccl":
                    cs.best_allreduce(comm, res_buf, o2, key)
                else:
                    key.copy_(res_buf[19:20] * (1 << 32) + (0xFFFFFFFF - (o2 + res_buf[17:18])))
                    comm.max_(key)

            for _ in range(3):
                ransac_strong_run()
            torch.cuda.synchronize()
            rs_el, rs_ev, rs_prof = timed(ransac_strong_run, args.ransac_steps, (K_SC, K_COMM))
            kc, kid = D.unpack_best_key(int(key.item()))
            ransac_strong = {"value": H * args.ransac_steps / rs_el, "ms_per_run": rs_el / args.ransac_steps * 1e3,
                             "score_ms_per_run": max_over_ranks(rs_prof[K_SC][0] / args.ransac_steps),
                             "exchange_ms_per_run": (max_over_ranks(rs_prof[K_COMM][0] / args.ransac_steps)
                                                     if rs_prof[K_COMM][1] else None),
                             "ms_per_run_with_events": rs_ev / args.ransac_steps * 1e3,
                             "hyps_per_run": H, "hyps_on_rank": c2, "best_id": kid, "best_count": kc,
                             "workload": f"cfg2 fixed batch: {H} hypotheses split over {world} GPUs, MAX key"}
        # cfg2's secondary workload (the GUI default _visualize_matcher.py:168):
        # noise_ratio 2.0 on the same pair (ransac.py:89-99 after np.random.seed(3): Nc = 3e5, the
        # set tests/golden/ransac_cfg2_full.npz pins), 1e5 hypotheses, the GUI's comparator
        # (evaluate_inlier_ratio_fast, Σd² < (1.5·v)²), seed 42, no early stop
        from matcher.ransac import inject_noise

        np.random.seed(3)
        corr3 = inject_noise(np.asarray(corr), len(rs_src), len(rs_tgt), 2.0)
        cs3 = CorrSet(rs_src, rs_tgt, corr3)
        p3 = RansacParams(max_iter=H, seed=42, thr=thr * thr, mode=_lib.SCORE_SQUARED, early_stop=False,
                          hyp0=rank * H)
        res3 = torch.zeros(RESULT_WORDS, dtype=torch.int64, device=dev)

        def ransac3_run():
            cs3.run_async(p3, res3)
            if multi:
                if comm_name == "libm3d-rccl":
                    cs3.best_allreduce(comm, res3, rank * H, key)
                else:
                    key.copy_(res3[19:20] * (1 << 32) + (0xFFFFFFFF - (rank * H + res3[17:18])))
                    comm.max_(key)

        for _ in range(3):
            ransac3_run()
        torch.cuda.synchronize()
        rel3, rel3_ev, prof3 = timed(ransac3_run, args.ransac_steps, (K_SC, K_KB))
        out3 = RansacOutcome.from_device(res3, len(corr3))
        sc3_avg = max_over_ranks(prof3[K_SC][0] / max(prof3[K_SC][1], 1))
        pairs3 = len(corr3) * H / max(prof3[K_SC][1] // args.ransac_steps, 1)
        sc3_algo = SCORE_FLOP_PER_PAIR * pairs3 / (sc3_avg * 1e-3) / 1e12
        ransac_nc3e5 = {
            "metric": "RANSAC hypotheses/sec (cfg2 secondary: noise_ratio 2.0, Nc=3e5, a1+a3, no early stop)",
            "value": world * H * args.ransac_steps / rel3, "unit": "hyp/s",
            "ms_per_run": rel3 / args.ransac_steps * 1e3, "nc": len(corr3), "hyps_per_gpu": H,
            "best_fitness": out3.fitness, "best_index": out3.best_index,
            "roofline": {"bound": "mfma", "kernel": "score_mfma_kernel", "achieved": sc3_algo,
                         "peak": MFMA_F16_PEAK_TF, "unit": "TFLOP/s", "frac": sc3_algo / MFMA_F16_PEAK_TF,
                         "avg_launch_ms": sc3_avg, "pairs_per_launch": pairs3,
                         "flop_per_pair": SCORE_FLOP_PER_PAIR,
                         "mfma_issue_frac": SCORE_MFMA_FLOP_PER_PAIR * pairs3 / (sc3_avg * 1e-3) / 1e12
                         / MFMA_F16_PEAK_TF},
        }
        del cs3
        ransac = {
            "metric": "RANSAC hypotheses/sec (cfg2: Nc=1e5, a1+a2, no early stop)",
            "value": world * H * args.ransac_steps / rel, "unit": "hyp/s",
            "ms_per_run": rel / args.ransac_steps * 1e3,
            "ms_per_run_with_kernel_events": rel_ev / args.ransac_steps * 1e3,
            "hyps_per_gpu": H, "nc": nc, "best_fitness": out.fitness,
            "roofline": {"bound": "mfma", "kernel": "score_mfma_kernel", "achieved": sc_algo,
                         "peak": MFMA_F16_PEAK_TF, "unit": "TFLOP/s", "frac": sc_algo / MFMA_F16_PEAK_TF,
                         "traffic": pmc_traffic("score_mfma_kernel")[0],
                         "avg_launch_ms": sc_avg, "launches": sc_n, "flop_per_pair": SCORE_FLOP_PER_PAIR,
                         "pairs_per_launch": pairs, "mfma_issued_tflops": sc_issued,
                         "mfma_issue_frac": sc_issued / MFMA_F16_PEAK_TF,
                         "vs_fp32_valu_roof": sc_algo / VALU_FP32_PEAK_TF,
                         "note": "27-flop/pair algorithmic rate / dense FP16 MFMA peak (the residuals "
                                 "run on the matrix pipe, DESIGN.md 3.2a)"},
            "kabsch_avg_launch_ms": kb_ms / max(kb_n, 1),
            "strong": ransac_strong,
            "nc3e5": ransac_nc3e5,
        }

    # ------------------------------------------------------------------ drop-in per-call path
    ransac_api = None
    if rank == 0 and world == 1 and not args.no_ransac_api:
        ransac_api = bench_ransac_api(args)

    # ------------------------------------------------------------------ cfg4: STL -> PLY -> register
    cfg4 = None
    if rank == 0 and world == 1 and not args.no_cfg4:
        cfg4 = bench_cfg4(args)

    # ------------------------------------------------------------------ CPU baseline
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(src, tgt_all[:nt], nrm_all[:nt], r, args, ransac is not None)

    if args.config == "cfg3":
        head = dict(metric="ICP iterations/sec (cfg3: 1M<->1M, target shard over N GPUs)",
                    value=cfg3["value"], unit=cfg3["unit"], scaling="strong", steps=args.cfg3_steps,
                    ms_per_step=cfg3["ms_per_iteration"] * args.cfg3_iters,
                    workload=cfg3["workload"], roofline=cfg3["roofline"])
    else:
        head = dict(metric="ICP iterations/sec + RANSAC hypotheses/sec, 100k↔100k pts, 1/2/4/8 GPU",
                    value=cfg1["value"], unit="ICP iter/s (100k src x 100k tgt per GPU)", scaling="weak",
                    steps=args.steps, ms_per_step=cfg1["ms_per_step"], workload=cfg1["workload"],
                    roofline=cfg1["roofline"])
    line = {
        "metric": head["metric"],
        "value": head["value"],
        "unit": head["unit"],
        "n_gpus": world,
        "steps": head["steps"],
        "warmup": args.warmup,
        "ms_per_step": head["ms_per_step"],
        "higher_is_better": True,
        "scaling": head["scaling"],
        "vs_baseline": None,
        "dtype": "fp16-split MFMA NN screen + fp32 scan, exact fp64 NN decision, fp64 terms/solve",
        "data": "synthetic (m3d.synth: asymmetric closed surface, extent ~10, analytic normals)",
        "config": {"workload": head["workload"], "ns": ns, "nt_per_gpu": nt, "icp_iterations_per_step": iters,
                   "max_corr": r, "parallelism": "single" if not multi else f"{mode1}-shard x{world}",
                   "comm": comm_name, "comm_ranks": comm_ranks},
        "roofline": head["roofline"],
        "ms_per_step_with_kernel_events": cfg1["ms_per_step_with_kernel_events"],
        "cfg1": {k: v for k, v in cfg1.items() if k != "roofline"} if args.config == "cfg3" else None,
        "icp_grid": icp_grid,
        "cfg1_strong": cfg1_strong,
        "cfg1_cold": cfg1_cold,
        "cfg3": (cfg3 if args.config != "cfg3" or cfg3 is None
                 else {k: v for k, v in cfg3.items() if k != "roofline"}),
        "ransac": ransac,
        "ransac_api": ransac_api,
        "cfg4_synthetic": cfg4,
        "cpu_baseline": cpu,
        "check": cfg1["check"],
    }
    line["summary"] = build_summary(line)  # last: the part of the line a truncated tail keeps
    if rank == 0:
        print(json.dumps(line), flush=True)
    del comm
    if multi:
        dist.destroy_process_group()


def bench_cold(args, src, tgt, nrm, r, iters, reps=3, nns=("brute", "grid"), tag="cfg1"):
    """A pair from nothing on the device: per-stage wall ms (median of `reps` after one warm call;
    the refine leg median of `reps` as well)."""
    import numpy as np
    import torch

    from m3d import cache
    from m3d.core import Cloud, IcpLoop
    from matcher.icp import refine_registration
    from ply import Ply

    def once(nn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sc, tc = Cloud(src), Cloud(tgt, nrm)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        lp = IcpLoop(sc, tc, r, relative_fitness=-1.0, relative_rmse=-1.0, max_iteration=iters, nn=nn)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        lp.reset(np.eye(4))
        lp.steps(iters + 1)
        lp.result()
        t3 = time.perf_counter()
        return {"clouds_ms": (t1 - t0) * 1e3, "loop_create_ms": (t2 - t1) * 1e3,
                "iterations_ms": (t3 - t2) * 1e3, "total_ms": (t3 - t0) * 1e3}

    def refine():
        cache.clear()
        a, b = Ply.from_arrays(src), Ply.from_arrays(tgt, nrm)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = refine_registration(a, b, np.eye(4), 0.3)
        t1 = time.perf_counter()
        return (t1 - t0) * 1e3, res

    out = {"workload": f"{tag} pair {len(src)}<->{len(tgt)}, {iters} iterations, every device object built "
                       "inside the timed region"}
    for nn in nns:
        once(nn)
        runs = [once(nn) for _ in range(reps)]
        out[nn] = {k: float(np.median([x[k] for x in runs])) for k in runs[0]}
    refine()
    ms = []
    for _ in range(reps):
        t, res = refine()
        ms.append(t)
    out["refine_registration_ms"] = float(np.median(ms))
    out["refine_registration_iterations_note"] = ("Open3D default criteria (1e-6, 1e-6, 30), grid NN; "
                                                  f"fitness {res.fitness:.4f}")
    cache.clear()
    return out


def bench_cfg4(args):
    """cfg4 (BASELINE configs[4]) on generated scans: main.py:24-43's pipeline from STL files.
    Two tessellations of the synthetic surface (source moved by T^-1) as binary STL ->
    convert_stl-ply.py (m3d.plyio) -> Ply(path, 0.3) (ply.py:32-66, stages timed) ->
    global_registration (ransac.py:20-59) at the reference's iteration=30 and at 30000 ->
    refine_registration (icp.py:17-48).  One untimed pass on a small mesh first."""
    import tempfile

    import numpy as np
    import torch

    from m3d import plyio, synth
    from matcher.icp import refine_registration
    from matcher.ransac import global_registration
    from ply import Ply

    T = synth.random_rigid(31, rot_range=0.5, trans_range=0.5)
    out = {"pipeline": "STL -> convert_stl-ply.py -> Ply(0.3) -> global_registration -> refine_registration",
           "data": "generated meshes (m3d.synth.surface_mesh; the reference ships no scans)"}
    with tempfile.TemporaryDirectory() as d:
        for tag, nl in (("warm", 60), ("timed", args.cfg4_mesh)):
            v_s, f_s = synth.surface_mesh(nl, 2 * nl, seed=1)
            v_t, f_t = synth.surface_mesh(int(nl * 1.1), int(nl * 2.2), seed=2)
            plyio.write_stl(f"{d}/src.stl", synth.apply(np.linalg.inv(T), v_s), f_s)
            plyio.write_stl(f"{d}/tgt.stl", v_t, f_t)
            t0 = time.perf_counter()
            plyio.convert_stl_to_ply(f"{d}/src.stl", f"{d}/src.ply")
            plyio.convert_stl_to_ply(f"{d}/tgt.stl", f"{d}/tgt.ply")
            t_conv = time.perf_counter() - t0
            np.random.seed(0)
            src, tgt = Ply(f"{d}/src.ply", 0.3), Ply(f"{d}/tgt.ply", 0.3)
            res = {}
            for it in (30, 30000):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                coarse = global_registration(src, tgt, 0.3, iteration=it)
                t1 = time.perf_counter()
                fine = refine_registration(src, tgt, coarse.transformation, 0.3)
                t2 = time.perf_counter()
                res[it] = (coarse, fine, (t1 - t0) * 1e3, (t2 - t1) * 1e3)
            if tag == "warm":
                continue
            out.update({
                "src_vertices": len(v_s), "tgt_vertices": len(v_t),
                "src_down": len(src.pcd_down.points), "tgt_down": len(tgt.pcd_down.points),
                "convert_stl_ply_ms": t_conv * 1e3,
                "ply_stage_ms": {"src": src.stage_ms, "tgt": tgt.stage_ms},
            })
            for it, (coarse, fine, tg, tr) in res.items():
                out[f"iteration_{it}"] = {
                    "global_registration_ms": tg, "refine_registration_ms": tr,
                    "coarse_fitness": coarse.fitness, "fine_fitness": fine.fitness,
                    "fine_max_abs_err_vs_T_true": float(np.abs(fine.transformation - T).max())}
            out["reference_suite"] = reference_suite(src, tgt, f"{d}/src.ply", f"{d}/tgt.ply")
            # validation throughput: the same a6 call (EdgeLength 0.9 + Distance 0.45 checkers) with
            # a 0.03 validation radius below the 0.05 point noise, so no hypothesis reaches the
            # early exit and every checker-passing one of 30000 is validated (grid.hip
            # validate_kernel batches)
            from m3d import prep
            corr = prep.feature_correspondences(src.pcd_fpfh, tgt.pcd_fpfh, True)
            sp, tp = src.pcd_down.points, tgt.pcd_down.points
            kw = dict(edge_length=0.9, distance=0.45, max_iteration=30000, confidence=0.999)
            prep.ransac_on_correspondences(sp, tp, corr, 0.03, **kw)  # warm
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fr = prep.ransac_on_correspondences(sp, tp, corr, 0.03, **kw)
            dt = time.perf_counter() - t0
            out["validation_throughput"] = {
                "hypotheses": 30000, "validation_radius": 0.03, "correspondences": len(corr),
                "validations": fr.validations,
                "ms": dt * 1e3, "validations_per_s": fr.validations / dt,
                "point_evaluations_per_s": fr.validations * len(sp) / dt,
                "best_fitness": fr.fitness}
    return out


# benchmark_results.txt (the reference's own published profile; hardware and input sizes unstated)
PUBLISHED_MS = {"ply_loading": 791.23, "correspondence_computation": 8.98, "ransac_iteration": 0.76,
                "evaluate_inliers": 0.50, "compute_transformation": 0.24, "deep_copy": 3.83,
                "full_ransac": 21.12}


def reference_suite(src, tgt, src_path, tgt_path, iterations=100):
    """benchmark_ransac.py:223-275 (run_comprehensive_benchmark) through the drop-in, on the cfg4
    scans: ply_loading (two Ply(path) calls, :45-47), correspondence_computation
    (compute_feature_correspondences, :76-77), ransac_iteration / compute_transformation /
    evaluate_inliers (100 × a1 + a2, :105-113), deep_copy (copy.deepcopy(src.pcd), :141-142),
    full_ransac (global_registration, iteration 30, :193-194) — wall ms beside the published
    benchmark_results.txt (hardware and input sizes unstated there)."""
    import copy

    import numpy as np
    import torch

    from matcher.ransac import (compute_feature_correspondences, compute_step_transformation,
                                evaluate_inlier_ratio, global_registration)
    from ply import Ply

    def wall(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fn()
        torch.cuda.synchronize()
        return r, (time.perf_counter() - t0) * 1e3

    np.random.seed(0)
    (s2, t2), load_ms = wall(lambda: (Ply(src_path, 0.3), Ply(tgt_path, 0.3)))
    corres, corr_ms = wall(lambda: compute_feature_correspondences(s2, t2, noise_ratio=0.0))
    a = b = 0.0
    for _ in range(iterations):
        res, ta = wall(lambda: compute_step_transformation(s2, t2, corres))
        _, tb = wall(lambda: evaluate_inlier_ratio(s2, t2, corres, res.transformation, 0.3))
        a += ta
        b += tb
    cp = 0.0
    for _ in range(iterations):
        cp += wall(lambda: copy.deepcopy(s2.pcd))[1]
    full, full_ms = wall(lambda: global_registration(s2, t2, voxel_size=0.3, iteration=30))
    got = {"ply_loading": load_ms, "correspondence_computation": corr_ms,
           "ransac_iteration": (a + b) / iterations, "evaluate_inliers": b / iterations,
           "compute_transformation": a / iterations, "deep_copy": cp / iterations,
           "full_ransac": full_ms}
    return {"harness": "benchmark_ransac.py run_comprehensive_benchmark (voxel 0.3, noise 0.0, 100 "
                       "iterations, full RANSAC 30) through matcher/ply on the cfg4 scans",
            "points": [len(s2.pcd.points), len(t2.pcd.points)],
            "down_points": [len(s2.pcd_down.points), len(t2.pcd_down.points)],
            "correspondences": int(len(corres)), "full_ransac_fitness": float(full.fitness),
            "ms": got, "published_ms": PUBLISHED_MS,
            "speedup_vs_published": {k: PUBLISHED_MS[k] / v for k, v in got.items() if v > 0}}


def bench_ransac_api(args, budget_s=1.5):
    """benchmark_ransac.py:87-125 through the drop-in: per hypothesis one
    compute_step_transformation + one evaluate_inlier_ratio on Ply-likes (cfg0's 5k and cfg2's
    1e5 correspondences; legacy global RNG seeded 42).  Both cache key policies (m3d.cache)."""
    import numpy as np
    import torch

    from m3d import cache, synth
    from matcher import ransac as M
    from ply import Ply

    out = {"harness": "benchmark_ransac.py:87-125 (compute_step_transformation + evaluate_inlier_ratio "
                      "per hypothesis) through matcher.ransac",
           "reference_ms_survey_container_8_cores": {
               "5000": {"compute_step_transformation": 0.125, "evaluate_inlier_ratio": 0.423},
               "100000": {"compute_step_transformation": 1.43, "evaluate_inlier_ratio": 9.28}}}
    for nc in (5000, args.nc):
        s, t, corr, _ = synth.ransac_pair(nc, seed=42)
        src, tgt = Ply.from_arrays(s), Ply.from_arrays(t)
        for pol in ("content", "identity"):
            cache.set_policy(pol)
            cache.clear()
            np.random.seed(42)
            for _ in range(3):  # pack + first calls
                res = M.compute_step_transformation(src, tgt, corr)
                M.evaluate_inlier_ratio(src, tgt, corr, res.transformation, 0.3)
            torch.cuda.synchronize()
            a = b = 0.0
            n = 0
            t_end = time.perf_counter() + budget_s
            while time.perf_counter() < t_end or n < 20:
                t0 = time.perf_counter()
                res = M.compute_step_transformation(src, tgt, corr)
                t1 = time.perf_counter()
                M.evaluate_inlier_ratio(src, tgt, corr, res.transformation, 0.3)
                t2 = time.perf_counter()
                a += t1 - t0
                b += t2 - t1
                n += 1
            out[f"{nc}_{pol}"] = {"compute_step_transformation_ms": a / n * 1e3,
                                  "evaluate_inlier_ratio_ms": b / n * 1e3,
                                  "hyps_per_s": n / (a + b), "hypotheses": n}
    cache.set_policy("content")
    cache.clear()
    return out


def cpu_baseline(src, tgt, nrm, r, args, with_ransac):
    """Oracle ('port') on the host: bounded samples of the same two workloads."""
    import numpy as np
    from scipy.spatial import cKDTree

    sys.path.insert(0, str(ROOT / "oracle"))
    import icp_oracle as I
    import ransac_oracle as O
    from m3d import synth

    cores, detail = host_cores()
    # ICP: Open3D-semantics iterations (KD-tree built once, like RegistrationICP)
    tree = cKDTree(tgt)
    T = np.eye(4)
    pcd = I.initial_points(T, src)
    n_it = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_budget and n_it < 200:
        d, j = tree.query(pcd, k=1, workers=cores)
        ok = d * d < r * r
        corr = np.stack([np.nonzero(ok)[0], j[ok]], axis=1)
        upd = I.point_to_plane_update(pcd, tgt, nrm, corr)
        T = upd @ T
        pcd = I.transform_points(upd, pcd)  # RegistrationICP: pcd.Transform(update)
        n_it += 1
    icp_el = time.perf_counter() - t0
    out = {"value": n_it / icp_el, "unit": "ICP iter/s (100k src x 100k tgt)", "cores": cores,
           "cores_detail": detail, "kind": "port",
           "sample": f"{n_it} Open3D-semantics point-to-plane iterations on the cfg1 pair "
                     f"(oracle/icp_oracle.py: scipy cKDTree workers={cores}, numpy fp64; "
                     "KD-tree build excluded)"}
    if with_ransac:
        src_r, tgt_r, corr_r, _ = synth.ransac_pair(args.nc, seed=42)
        rng = np.random.RandomState(42)
        n_h = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < args.cpu_budget and n_h < 5000:
            Th, _, _ = O.compute_step_transformation(src_r, tgt_r, corr_r, rng=rng)
            O.evaluate_inlier_ratio(src_r, tgt_r, corr_r, Th, 0.3)
            n_h += 1
        rel = time.perf_counter() - t0
        out["ransac"] = {"value": n_h / rel, "unit": "hyp/s", "cores": 1, "kind": "port",
                         "sample": f"{n_h} hypotheses of benchmark_ransac.py's loop (a1 + a2, numpy fp64, "
                                   f"legacy RNG permutation sampling) at Nc={args.nc}"}
    return out


if __name__ == "__main__":
    main()
