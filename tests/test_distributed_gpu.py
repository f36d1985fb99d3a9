"""Multi-process data parallelism on the GPU path: one rank per device, segmented HIP-graph
capture cut at the collectives, bucketed gradient all-reduce overlapped with the backward.

The GPU box has one MI355X and RCCL refuses two ranks on one GPU, so the ranks here share the
GPU over gloo (``LJS_DIST_BACKEND=gloo``): every framework code path of an N-GPU run
(DistComm, the async grad reducer, graph segments, joins) executes; only the transport
differs from RCCL over xGMI.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "scripts", "dp_check.py")


def _run(tmp_path, world, capture, steps=3, port=29517, wire="bf16", mesh=None, gb=4, extra_env=None, tag=""):
    out = str(tmp_path / f"w{world}_c{capture}_{wire}_{mesh}{tag}.npz")
    env = dict(os.environ, PYTHONPATH=ROOT, LJS_PLATFORM="gpu", LJS_DIST_BACKEND="gloo", LJS_GRAD_COMM_DTYPE=wire,
               **(extra_env or {}))
    env.pop("LJS_NUM_DEVICES", None)
    if world == 1:
        cmd = [sys.executable, SCRIPT, out, str(steps), str(int(capture)), str(gb)]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={port + world + 10 * int(capture)}", SCRIPT, out,
               str(steps), str(int(capture)), str(gb)] + ([mesh] if mesh else [])
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return np.load(out)


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_dp2_graph_matches_single_process(tmp_path, wire):
    """fp32 wire: DP == single process to f32 reassociation, except that Adam's first steps move
    each weight by ~lr times the SIGN of its gradient: a near-zero gradient whose reassociated
    sum (half-batch weight-gradient split-K slabs, then the all-reduce) flips sign moves that
    weight by up to 2 lr per step -- a handful of elements of the 0.33 M, bounded by 3 steps x
    2 lr.  bf16 wire (the reference's own bf16 gradient all-reduce): the same with bf16-rounded
    sums, so more such elements."""
    ref = _run(tmp_path, 1, False, wire=wire)
    eager = _run(tmp_path, 2, False, port=29537 if wire == "bf16" else 29517, wire=wire)
    graph = _run(tmp_path, 2, True, port=29537 if wire == "bf16" else 29517, wire=wire)
    assert int(graph["step"]) == 3 and int(eager["step"]) == 3
    for k in ref.files:
        if k == "step":
            continue
        if wire == "fp32":
            diff = np.abs(eager[k] - ref[k])
            assert diff.max() <= 6e-3 + 1e-6, (k, diff.max())
            assert np.mean(diff > 2e-4 + 2e-3 * np.abs(ref[k])) < 1e-4, (k, np.mean(diff > 2e-4))
        else:
            diff = np.abs(eager[k] - ref[k])
            assert diff.max() <= 6e-3 + 1e-6, (k, diff.max())
            assert np.mean(diff > 2e-4 + 2e-3 * np.abs(ref[k])) < 5e-3, (k, np.mean(diff > 2e-4))
        np.testing.assert_allclose(graph[k], eager[k], rtol=1e-5, atol=1e-6, err_msg=f"graph {k}")


@pytest.mark.parametrize("world,mesh", [(2, "1x2"), (4, "2x2")])
def test_2d_layout_matches_single_process(tmp_path, world, mesh):
    """The reference's 2-D layout (sequence and Q/K/V weights over 'model', batch over 'data') on
    ranks sharing the GPU: seq-major activations, K/V / head gathers and the out-projection
    all-to-all as whole-block collectives (no pack kernels) - same parameters as one process."""
    ref = _run(tmp_path, 1, False, wire="fp32", gb=4)
    got = _run(tmp_path, world, False, port=29557 + world, wire="fp32", mesh=mesh, gb=4)
    for k in ref.files:
        if k == "step":
            continue
        diff = np.abs(got[k] - ref[k])
        assert diff.max() <= 6e-3 + 1e-6, (k, diff.max())
        assert np.mean(diff > 2e-4 + 2e-3 * np.abs(ref[k])) < 5e-3, (k, np.mean(diff > 2e-4))


def test_2d_layout_graph_matches_eager(tmp_path):
    """The 2-D layout under a segmented HIP-graph capture cut at its gloo collectives -- some of
    them issued where the layout forks a side stream (prefetched gathers) -- replays to the eager
    run's parameters.  (Before the capture's cuts were made stream-safe this raised "Capture must
    end on the same stream it began on": profiles/r6ab_gloo_multirank_lines.txt, the 2-D secondary.)"""
    eager = _run(tmp_path, 2, False, port=29621, wire="fp32", mesh="1x2", gb=4, tag="e")
    graph = _run(tmp_path, 2, True, port=29641, wire="fp32", mesh="1x2", gb=4, tag="g")
    assert int(graph["step"]) == 3 and int(eager["step"]) == 3
    for k in eager.files:
        np.testing.assert_allclose(graph[k], eager[k], rtol=1e-5, atol=1e-6, err_msg=f"graph {k}")


def test_dp2_early_input_cast_bit_exact(tmp_path):
    """LJS_PRECAST=join: in a data-parallel multi-step graph the next step's input cast is queued
    before the gradient all-reduce join instead of in that step's forward -- the same bf16 values,
    so the trained parameters are bit-identical to the in-forward cast."""
    kw = dict(steps=4, gb=32, wire="fp32")
    a = _run(tmp_path, 2, True, port=29561, extra_env={"LJS_CHECK_MULTI": "2", "LJS_PRECAST": "join"}, tag="j", **kw)
    b = _run(tmp_path, 2, True, port=29571, extra_env={"LJS_CHECK_MULTI": "2", "LJS_PRECAST": "0"}, tag="o", **kw)
    assert int(a["step"]) == 4 and int(b["step"]) == 4
    assert int(a["precast_taken"]) > 0 and int(b["precast_taken"]) == 0
    for k in a.files:
        if k != "precast_taken":
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
