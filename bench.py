#!/usr/bin/env python3
"""Benchmark: ICP iterations/s (cfg1) + RANSAC hypotheses/s (cfg2) on synthetic 100k↔100k pairs.

BASELINE.json metric "ICP iterations/sec + RANSAC hypotheses/sec, 100k↔100k pts, 1/2/4/8 GPU".

* step (the timed unit) = one full cfg1 ICP run: 100k source ↔ 100k target points per GPU,
  50 point-to-plane iterations (convergence disabled → exactly 50 updates, 51 NN evaluations),
  brute-force radius-bounded NN (r = 0.4·0.3), fp64 terms/solve, all device resident.
  value = ICP iterations/s summed over ranks (each rank does one 100k×100k block per
  iteration; N>1 is weak scaling).  N>1 follows the north-star's rule: the TARGET is sharded
  (100k targets per rank, sources replicated, RCCL MIN of the packed NN keys + SUM of the 32
  estimation terms per iteration — the cfg3 protocol) only when the cloud would not fit one
  GPU's HBM; otherwise the sources are sharded (100k per rank) against the replicated target
  with one RCCL SUM of the terms per iteration.  `--shard target|source` forces either.
* "ransac": cfg2 — benchmark_ransac.py's loop (a1 sample + Kabsch, a2 ‖d‖ < 1.5·v scoring) at
  Nc = 1e5, H = 1e5 hypotheses per GPU, counter sampler seed 42, no early stop; N>1 shards the
  hypothesis ids and all-reduces MAX of the packed (count, ~id) best key.  Its roofline prices
  score_mfma_kernel (three v_mfma_f32_32x32x16_f16 per 32×32 (correspondence, hypothesis)
  block = 96 flop per pair) against the FP16 MFMA peak; the 27-flop algorithmic figure is given
  beside it against the FP32 vector roof.
* roofline: dominant kernel = the ICP NN scan (nn_mfma_kernel), timed with HIP events recorded
  by the library on the launch stream around every NN launch during a second timed pass of the
  same K steps (an event record costs ~4 us between dependent kernels — tools/loop_overhead.py —
  so `value` comes from the pass without them; both step times are in the line).  Its
  screen key |t|² − 2q·t is a rank-4 contraction run on the matrix cores as one
  v_mfma_f32_32x32x16_f16 per 32×32 (target, query) block: 16 fp16 MACs = 32 flop per pair
  (K = 16 fp16 hi/lo split terms, 11 non-zero), so bound = "mfma" against the
  dense FP16 MFMA peak 2.5 PFLOP/s, achieved = 32 flop × Ns × Nt / launch time.  The SURVEY's
  8-flop-per-pair algorithmic figure is reported beside it against the FP32 vector roof
  (157.3 TFLOP/s) that a VALU implementation is bounded by.  traffic = HBM bytes per launch
  from the committed rocprofv3 PMC summary (profiles/), or null.
* "icp_grid": the same cfg1 workload with the radius-bounded uniform-grid NN (SURVEY §8(f)
  rank 1; identical correspondences, tests/test_gpu_icp.py) — HBM/latency-bound, so its
  roofline is priced in GB/s on 28·Ns + 16·Nt algorithmic bytes per launch (query float4 +
  visit order + key write, each target read once).
* cpu_baseline (rank 0, N = 1): the oracle restatement (oracle/icp_oracle.py: scipy cKDTree on
  16 threads + numpy point-to-plane) timed on a bounded sample of the same workload.
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
NN_FLOP_PER_PAIR = 8        # 3 sub + 1 mul + 2 FMA (SURVEY §8(d), fp32 VALU formulation)
NN_MFMA_FLOP_PER_PAIR = 32  # 16 fp16 MACs per (target, query) pair in v_mfma_f32_32x32x16_f16
SCORE_FLOP_PER_PAIR = 27    # 9 FMA transform + 3 sub + (1 mul + 2 FMA) + 1 cmp
SCORE_MFMA_FLOP_PER_PAIR = 96  # 3 x v_mfma_f32_32x32x16_f16 (16 fp16 MACs each) per pair
CPU_THREADS = 16            # the GPU box's CPU share per GPU


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--ns", type=int, default=100_000)
    ap.add_argument("--nt", type=int, default=100_000, help="target points per GPU")
    ap.add_argument("--icp-iters", type=int, default=50)
    ap.add_argument("--nc", type=int, default=100_000)
    ap.add_argument("--hyps", type=int, default=100_000, help="RANSAC hypotheses per GPU per run")
    ap.add_argument("--ransac-steps", type=int, default=3)
    ap.add_argument("--no-ransac", action="store_true")
    ap.add_argument("--ransac-warmup-s", type=float, default=0.5,
                    help="untimed RANSAC runs for at least this long before the timed ones")
    ap.add_argument("--no-grid", action="store_true")
    ap.add_argument("--shard", choices=["auto", "target", "source"], default="auto",
                    help="N>1 ICP sharding: target (RCCL MIN of the NN keys + SUM of the terms), "
                         "source (target replicated, SUM of the terms only), or auto: the "
                         "north-star's rule -- shard the target only when it would not fit one "
                         "GPU's HBM budget (M3D_TARGET_SHARD_BYTES, default 64 GiB), else source")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=8.0, help="seconds per CPU baseline leg")
    return ap.parse_args()


def pmc_traffic(kernel_substr: str):
    """HBM bytes per launch from the newest committed PMC summary (profiles/pmc_*.json)."""
    files = sorted((ROOT / "profiles").glob("pmc_*.json"))
    for f in reversed(files):
        try:
            d = json.loads(f.read_text())
        except Exception:
            continue
        for k, v in d.get("kernels", {}).items():
            if kernel_substr in k and v.get("hbm_bytes_per_launch") is not None:
                return float(v["hbm_bytes_per_launch"]), f.name
    return None, None


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # M3D_BENCH_SAME_DEVICE=1 + M3D_BENCH_BACKEND=gloo: every rank on cuda:0 over gloo — a
        # functional rehearsal of the N > 1 path on a one-GPU box (tools/gpu_multi_rehearsal.sh);
        # the real runs are one rank per GPU over RCCL ("nccl")
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
    from m3d.core import Cloud, CorrSet, IcpLoop, RansacParams, context

    ctx = context()

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # ------------------------------------------------------------------ cfg1: ICP
    ns, nt, iters = args.ns, args.nt, args.icp_iters
    r = 0.4 * 0.3
    if args.shard == "auto":
        # north_star: "shards the target cloud ... with an RCCL all-reduce of per-shard
        # (min_dist, argmin) ... only for clouds large enough to saturate one GPU's HBM"; a
        # replicated cloud costs 64 B per point
        budget = float(os.environ.get("M3D_TARGET_SHARD_BYTES", 64 * 2**30))
        args.shard = "target" if 64.0 * nt * world > budget else "source"
    source_shard = world > 1 and args.shard == "source"
    if source_shard:  # weak scaling: ns sources per rank against the whole (replicated) target
        src_all, tgt_all, nrm_all, T_true = synth.icp_pair(ns * world, nt, seed=0)
        src = src_all[rank * ns:(rank + 1) * ns]
        off = 0
        tgt_c = Cloud(tgt_all, nrm_all)
    else:  # target-sharded: nt targets per rank, sources replicated
        src, tgt_all, nrm_all, T_true = synth.icp_pair(ns, nt * world, seed=0)
        off = rank * nt
        # one fp32 frame for every shard (the whole target's mean): keys compare bit for bit
        # across ranks, and non-owning ranks start from a distance bound (m3d_cloud_create_framed)
        tgt_c = Cloud(tgt_all[off:off + nt], nrm_all[off:off + nt], center=tgt_all.mean(axis=0))
    src_c = Cloud(src)
    keys = torch.empty(ns, dtype=torch.int64, device=dev)
    claim = torch.empty(ns, dtype=torch.int32, device=dev)
    sums = torch.empty(32, dtype=torch.float64, device=dev)

    def time_icp(nn: str):
        loop = IcpLoop(src_c, tgt_c, r, relative_fitness=-1.0, relative_rmse=-1.0, max_iteration=iters,
                       nn=nn)
        if source_shard:
            loop.set_source_total(ns * world)

        def icp_run():
            loop.reset(np.eye(4))
            if world == 1:
                loop.steps(iters + 1)  # the library enqueues the 51 iterations natively
                return
            for _ in range(iters + 1):
                if source_shard:  # keys stay inside the loop object: no copies
                    loop.shard_nn(0, None)
                    loop.shard_terms(0, None, None, sums)
                    dist.all_reduce(sums, op=dist.ReduceOp.SUM)
                    loop.solve(sums)
                else:
                    loop.shard_nn(off, keys)
                    dist.all_reduce(keys, op=dist.ReduceOp.MIN)
                    loop.shard_claim(keys, claim)
                    dist.all_reduce(claim, op=dist.ReduceOp.MIN)
                    loop.shard_terms(off, keys, claim, sums)
                    dist.all_reduce(sums, op=dist.ReduceOp.SUM)
                    loop.solve(sums)

        def timed(events: bool):
            ctx.profile(events)
            ctx.profile_read(_lib.KERNEL_NN)
            ctx.profile_read(_lib.KERNEL_TERMS)
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                icp_run()
            torch.cuda.synchronize()
            barrier()
            el = max_over_ranks(time.perf_counter() - t0)
            nn_ms, nn_n = ctx.profile_read(_lib.KERNEL_NN)
            terms_ms, terms_n = ctx.profile_read(_lib.KERNEL_TERMS)
            ctx.profile(False)
            return el, nn_ms, nn_n, terms_ms, terms_n

        for _ in range(args.warmup):
            icp_run()
        torch.cuda.synchronize()
        # value: the K steps with nothing else on the stream.  Kernel durations: the same K steps
        # again with the library's HIP events around every NN and terms launch (each event record
        # costs ~4 us of stream time between dependent kernels: tools/loop_overhead.py).
        el, _, _, _, _ = timed(False)
        el_ev, nn_ms, nn_n, terms_ms, terms_n = timed(True)
        return (el, max_over_ranks(nn_ms / max(nn_n, 1)), nn_n, terms_ms / max(terms_n, 1),
                loop.result(), el_ev)

    el, nn_avg_ms, nn_n, terms_avg_ms, res, el_ev = time_icp("brute")
    icp_value = world * iters * args.steps / el
    nn_flop = NN_MFMA_FLOP_PER_PAIR * ns * nt
    achieved_tf = nn_flop / (nn_avg_ms * 1e-3) / 1e12
    algo_tf = NN_FLOP_PER_PAIR * ns * nt / (nn_avg_ms * 1e-3) / 1e12
    err = float(np.abs(res.transformation - T_true).max())

    # ------------------------------------------------------------------ cfg1 with the grid NN
    icp_grid = None
    if not args.no_grid:
        tg0 = time.perf_counter()
        IcpLoop(src_c, tgt_c, r, max_iteration=0, nn="grid")  # builds both clouds' grids once
        torch.cuda.synchronize()
        build_ms = (time.perf_counter() - tg0) * 1e3
        gel, g_ms, g_n, g_terms_ms, gres, gel_ev = time_icp("grid")
        g_bytes = 28 * ns + 16 * nt
        g_gbs = g_bytes / (g_ms * 1e-3) / 1e9
        icp_grid = {
            "metric": "ICP iterations/sec (cfg1 workload, uniform-grid radius NN)",
            "value": world * iters * args.steps / gel, "unit": "ICP iter/s (100k src x 100k tgt per GPU)",
            "ms_per_step": gel / args.steps * 1e3, "grid_build_ms": build_ms,
            "ms_per_step_with_kernel_events": gel_ev / args.steps * 1e3,
            "same_result_as_brute": bool(np.array_equal(gres.transformation, res.transformation)),
            "roofline": {"bound": "hbm", "kernel": "grid_nn_kernel", "achieved": g_gbs,
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": g_gbs / HBM_PEAK_GBS,
                         "traffic": pmc_traffic("grid_nn_kernel")[0], "avg_launch_ms": g_ms,
                         "launches": g_n, "bytes_per_launch": g_bytes,
                         "terms_avg_launch_ms": g_terms_ms},
        }

    # ------------------------------------------------------------------ cfg2: RANSAC
    ransac = None
    if not args.no_ransac:
        nc, H = args.nc, args.hyps
        rs_src, rs_tgt, corr, _ = synth.ransac_pair(nc, seed=42)
        cs = CorrSet(rs_src, rs_tgt, corr)
        thr = 0.3 * 1.5
        params = RansacParams(max_iter=H, seed=42, thr=thr, mode=_lib.SCORE_NORM, early_stop=False,
                              hyp0=rank * H)

        from m3d.core import RESULT_WORDS, RansacOutcome
        res_buf = torch.zeros(RESULT_WORDS, dtype=torch.int64, device=dev)

        def ransac_run():
            # enqueued without a host round trip (m3d_ransac_run_async): runs go back to back
            cs.run_async(params, res_buf)
            if world > 1:  # best over ranks: highest count, lowest global id (device-side key)
                key = (res_buf[19:20] * (1 << 32) + (0xFFFFFFFF - (rank * H + res_buf[17:18])))
                dist.all_reduce(key, op=dist.ReduceOp.MAX)
            return res_buf

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

        def ransac_timed(events: bool):
            ctx.profile(events)
            ctx.profile_read(_lib.KERNEL_SCORE)
            ctx.profile_read(_lib.KERNEL_KABSCH)
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.ransac_steps):
                out = ransac_run()
            torch.cuda.synchronize()
            barrier()
            el = max_over_ranks(time.perf_counter() - t0)
            sc = ctx.profile_read(_lib.KERNEL_SCORE)
            kb = ctx.profile_read(_lib.KERNEL_KABSCH)
            ctx.profile(False)
            return el, sc, kb, RansacOutcome.from_device(out, nc)

        rel, _, _, out = ransac_timed(False)  # value: no events on the stream
        rel_ev, (sc_ms, sc_n), (kb_ms, kb_n), _ = ransac_timed(True)  # kernel durations
        sc_avg = max_over_ranks(sc_ms / max(sc_n, 1))
        hyps_per_launch = H / max(sc_n // args.ransac_steps, 1)
        sc_tf = SCORE_MFMA_FLOP_PER_PAIR * nc * hyps_per_launch / (sc_avg * 1e-3) / 1e12
        sc_algo_tf = SCORE_FLOP_PER_PAIR * nc * hyps_per_launch / (sc_avg * 1e-3) / 1e12
        ransac = {
            "metric": "RANSAC hypotheses/sec (cfg2: Nc=1e5, a1+a2, no early stop)",
            "value": world * H * args.ransac_steps / rel, "unit": "hyp/s",
            "ms_per_run": rel / args.ransac_steps * 1e3,
            "ms_per_run_with_kernel_events": rel_ev / args.ransac_steps * 1e3,
            "hyps_per_gpu": H, "nc": nc,
            "best_fitness": out.fitness,
            "roofline": {"bound": "mfma", "kernel": "score_mfma_kernel", "achieved": sc_tf,
                         "peak": MFMA_F16_PEAK_TF, "unit": "TFLOP/s", "frac": sc_tf / MFMA_F16_PEAK_TF,
                         "avg_launch_ms": sc_avg, "launches": sc_n,
                         "flop_per_pair": SCORE_MFMA_FLOP_PER_PAIR,
                         "algorithmic_27flop_per_pair_tflops": sc_algo_tf,
                         "vs_fp32_valu_roof": sc_algo_tf / VALU_FP32_PEAK_TF},
            "kabsch_avg_launch_ms": kb_ms / max(kb_n, 1),
        }

    # ------------------------------------------------------------------ CPU baseline
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(src, tgt_all[:nt], nrm_all[:nt], r, args, ransac is not None)

    traffic, traffic_src = pmc_traffic("nn_mfma_kernel")
    line = {
        "metric": "ICP iterations/sec + RANSAC hypotheses/sec, 100k↔100k pts, 1/2/4/8 GPU",
        "value": icp_value,
        "unit": "ICP iter/s (100k src x 100k tgt per GPU)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": el / args.steps * 1e3,
        "ms_per_step_with_kernel_events": el_ev / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f16-split MFMA NN screen (exact f32 NN result) + f64 terms/solve",
        "data": "synthetic (m3d.synth: asymmetric closed surface, extent ~10, analytic normals)",
        "config": {"workload": "cfg1: 100k<->100k synthetic pair, 50 point-to-plane ICP iterations, "
                               "brute-force NN (r=0.12), 1 GPU" if world == 1 else
                               (f"cfg1 per GPU, sources sharded over {world} GPUs, target replicated (RCCL SUM terms)"
                                if source_shard else
                                f"cfg1 per GPU, target sharded over {world} GPUs (RCCL MIN keys + SUM terms)"),
                   "ns": ns, "nt_per_gpu": nt, "icp_iterations_per_step": iters, "max_corr": r,
                   "parallelism": "single" if world == 1 else f"{args.shard}-shard x{world}"},
        "roofline": {"bound": "mfma", "kernel": "nn_mfma_kernel", "achieved": achieved_tf,
                     "peak": MFMA_F16_PEAK_TF, "unit": "TFLOP/s", "frac": achieved_tf / MFMA_F16_PEAK_TF,
                     "traffic": traffic, "traffic_source": traffic_src, "avg_launch_ms": nn_avg_ms,
                     "launches": nn_n, "flop_per_launch": nn_flop,
                     "flop_per_pair": NN_MFMA_FLOP_PER_PAIR,
                     "algorithmic_8flop_per_pair_tflops": algo_tf,
                     "vs_fp32_valu_roof": algo_tf / VALU_FP32_PEAK_TF,
                     "terms_avg_launch_ms": terms_avg_ms},
        "icp_grid": icp_grid,
        "ransac": ransac,
        "cpu_baseline": cpu,
        "check": {"icp_fitness": res.fitness, "icp_rmse": res.inlier_rmse, "max_abs_err_vs_T_true": err},
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(src, tgt, nrm, r, args, with_ransac):
    """Oracle ('port') on the host: bounded samples of the same two workloads."""
    import numpy as np
    from scipy.spatial import cKDTree

    sys.path.insert(0, str(ROOT / "oracle"))
    import icp_oracle as I
    import ransac_oracle as O
    from m3d import synth

    # ICP: Open3D-semantics iterations (KD-tree built once, like RegistrationICP)
    tree = cKDTree(tgt)
    T = np.eye(4)
    n_it = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < args.cpu_budget and n_it < 200:
        pcd = I.transform_points(T, src)
        d, j = tree.query(pcd, k=1, workers=CPU_THREADS)
        ok = d * d < r * r
        corr = np.stack([np.nonzero(ok)[0], j[ok]], axis=1)
        T = I.point_to_plane_update(pcd, tgt, nrm, corr) @ T
        n_it += 1
    icp_el = time.perf_counter() - t0
    out = {"value": n_it / icp_el, "unit": "ICP iter/s (100k src x 100k tgt)", "cores": CPU_THREADS,
           "kind": "port",
           "sample": f"{n_it} Open3D-semantics point-to-plane iterations on the cfg1 pair "
                     f"(oracle/icp_oracle.py: scipy cKDTree workers={CPU_THREADS}, numpy fp64; "
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
