"""The device block cache (api.cpp, ABI 12-13): stream-ordered reuse, trimming, and the
cloud-before-loop destruction order."""
import time

import numpy as np
import pytest

from m3d import synth
from m3d.core import Cloud, IcpLoop, context

pytestmark = pytest.mark.gpu


def test_reuse_waits_only_for_its_own_streams():
    """A cloud destroyed after work on stream A is reused by a new cloud on stream A while a
    long kernel runs on stream B (enqueued by torch, never by the library): the reuse makes A wait
    for A's release point only, so the new cloud is built while B is still busy (round 4 waited
    for the whole device with hipDeviceSynchronize), and the new cloud is correct."""
    import torch

    pts, _ = synth.surface_points(150_000, seed=4)
    c = Cloud(pts)
    del c  # its blocks go to the cache, marked after the current stream's work
    torch.cuda.synchronize()
    b = torch.cuda.Stream()
    x = torch.randn(8192, 8192, device="cuda")
    done_b = torch.cuda.Event()
    with torch.cuda.stream(b):
        for _ in range(60):
            x = x @ x * 1e-4
        done_b.record(b)
    t0 = time.perf_counter()
    c2 = Cloud(pts)  # same sizes: the cached blocks (synchronises its own stream only)
    dt = time.perf_counter() - t0
    busy = not done_b.query()
    torch.cuda.synchronize()
    t_b = time.perf_counter() - t0
    assert busy, f"the reuse waited for stream B (cloud {dt * 1e3:.1f} ms, B done after {t_b * 1e3:.1f} ms)"
    # the reused blocks hold the new cloud: NN against it is exact
    from m3d.core import nn1

    q = Cloud(pts[:2000] + 1e-3)
    i, _ = nn1(q, c2, np.eye(4), 0.05, nn="grid")
    assert (i.cpu().numpy() == np.arange(2000)).mean() > 0.99


def test_trim_gives_cached_blocks_back():
    ctx = context()
    pts, _ = synth.surface_points(50_000, seed=5)
    clouds = [Cloud(pts + k) for k in range(4)]
    del clouds
    freed = ctx.trim_block_cache()
    assert freed >= 4 * 50_000 * 24
    assert ctx.trim_block_cache() == 0


def test_loop_outlives_its_source_cloud():
    """Destroying the source cloud before its ICP loop (Python finalisers in reference cycles may
    run in that order) leaves the loop's Morton copy alive until the loop goes: the loop keeps
    stepping with the same bits, and destroying it afterwards frees the copy (no use after free)."""
    src, tgt, nrm, _ = synth.icp_pair(40_000, seed=31)
    s, t = Cloud(src), Cloud(tgt, nrm)
    kw = dict(relative_fitness=-1, relative_rmse=-1, max_iteration=12, nn="grid")
    ref = IcpLoop(s, t, 0.12, **kw)
    ref.reset(np.eye(4))
    ref.steps(13)
    want = ref.result()
    lp = IcpLoop(Cloud(src), t, 0.12, **kw)
    lp.reset(np.eye(4))
    lp.steps(5)
    lp.src.ctx.lib.m3d_cloud_destroy(lp.src.h)  # the C-level order the finalisers may take
    lp.src.h = None
    lp.steps(8)
    got = lp.result()
    np.testing.assert_array_equal(got.transformation, want.transformation)
    assert (got.fitness, got.inlier_rmse) == (want.fitness, want.inlier_rmse)
    del lp  # frees the orphaned Morton copy
    context().trim_block_cache()


def test_release_mark_covers_a_solve_only_sequence():
    """m3d_icp_solve (and m3d_icp_shard_claim) record their stream use, so a loop
    destroyed right after a solve queued behind long work on stream A goes back to the cache
    marked AFTER that solve: a new loop on stream B that reuses the block waits for it (round 5's
    mark was recorded at the previous touching call, before the solve, and B could take the block
    while the solve was still writing the loop state)."""
    import torch

    src, tgt, nrm, _ = synth.icp_pair(30_000, seed=8)
    s, t = Cloud(src), Cloud(tgt, nrm)
    kw = dict(relative_fitness=-1, relative_rmse=-1, max_iteration=5, nn="grid")
    a = torch.cuda.Stream()
    lp = IcpLoop(s, t, 0.12, **kw)
    sums = torch.zeros(32, dtype=torch.float64, device="cuda")
    with torch.cuda.stream(a):
        lp.reset(np.eye(4))
        lp.step()
    torch.cuda.synchronize()
    x = torch.randn(8192, 8192, device="cuda")
    done_a = torch.cuda.Event()
    with torch.cuda.stream(a):
        for _ in range(40):
            x = x @ x * 1e-4
        lp.solve(sums)  # the only library call after the long work on A
        done_a.record(a)
    del lp  # release marked after A's last touch: the solve
    b = torch.cuda.Stream()
    with torch.cuda.stream(b):
        lp2 = IcpLoop(s, t, 0.12, **kw)  # the cached block: creation waits for its mark
    assert done_a.query(), "the reused block was handed out before the solve on stream A finished"
    with torch.cuda.stream(b):
        lp2.reset(np.eye(4))
        lp2.steps(6)
        r = lp2.result()
    ref = IcpLoop(s, t, 0.12, **kw)
    ref.reset(np.eye(4))
    ref.steps(6)
    np.testing.assert_array_equal(r.transformation, ref.result().transformation)
