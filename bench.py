"""Headline benchmark: case6 sharded attention block train step (fwd + bwd + Adam).

Metric (BASELINE.json): "step-time ms + TFLOPS/GPU, case6 sharded attention block at 1/2/4/8
MI355X".  The model is the reference's FlaxAttention (``case6_attention.py:42-143``:
M=640, 8 heads x 64, bf16 compute, f32 params, Adam lr 1e-3) with the reference's
logical-axis rules; S=256 as in the reference.  Data is synthetic (random normal inputs,
random-init weights).  Work per GPU is fixed as N grows (weak scaling): the global batch is
``--batch-per-gpu x N`` sequences, and every mesh layout gives each GPU ``batch-per-gpu x S``
tokens.

Launch:
* ``python bench.py`` - one GPU.
* ``python bench.py --gpus N`` - spawns N rank processes (``torch.distributed.run``, one per
  GPU, RCCL over xGMI) BEFORE anything touches the GPU and exits with their status; fails if
  fewer than N GPUs are visible.  Under ``torchrun --nproc-per-node N bench.py --gpus N`` (the
  driver's launch) the ranks run directly; ``WORLD_SIZE`` must equal ``--gpus``.
* ``LJS_PLATFORM=cpu python bench.py --gpus N`` - the same N-rank job on gloo host ranks (CPU
  rehearsal of the multi-GPU code path; tests/test_bench_cpu.py).

``--mesh dp`` (default, (N,1)) or ``--mesh 2d`` ((N/2, 2): the reference's DP x TP layout,
``case6_attention.py:155-161,183-187``) or ``--mesh DxM``.  DP is the default because on
point-to-point xGMI the reference's TP layout (sequence over ``model``) moves activation-sized
K/V/head gathers and an all-to-all every step (~150 MB/GPU at 64x256 tokens), while DP moves
one 5 MB gradient all-reduce.

The step is a jitted, donated, HIP-graph-captured function; the timed region is K full steps
bracketed by barrier + device synchronize, and the reported time is the max over ranks.
Rank 0 prints one JSON line; ``value`` is the whole-job TFLOPS (summed over the N GPUs, the
driver's aggregate convention) and ``tflops_per_gpu`` the per-GPU rate the metric names.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "step-time ms + TFLOPS/GPU, case6 sharded attention block at 1/2/4/8 MI355X"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs (= ranks); default: WORLD_SIZE under torchrun, else 1")
    p.add_argument("--steps", type=int, default=48)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--min-warmup", type=int, default=int(os.environ.get("LJS_BENCH_MIN_WARM", "64")),
                   help="untimed steps in all before the timed region, at least: steps ~20-45 of a process run "
                        "under a measured 8-12 %% clock dip (a power-management transient: the in-kernel clock "
                        "probe of profiles/r6b_clock_ramp.md) and their kernels 5-7 %% slower; 64 untimed steps put "
                        "the timed region after it.  The JSON 'warmup' reports the total that ran")
    p.add_argument("--batch-per-gpu", type=int, default=int(os.environ.get("LJS_BENCH_BPG", "64")))
    p.add_argument("--seq", type=int, default=256)
    p.add_argument("--dim", type=int, default=640)
    p.add_argument("--heads", type=int, default=8)
    p.add_argument("--dim-head", type=int, default=64)
    p.add_argument("--mesh", default=os.environ.get("LJS_BENCH_MESH", "dp"),
                   help="dp: (N,1) data x model; 2d: (N/2, 2); or explicit 'DxM'")
    p.add_argument("--no-graph", action="store_true")
    p.add_argument("--mode", default="train", choices=["train", "fwd"])
    p.add_argument("--model", default="attention", choices=["attention", "layer", "ff", "fsdp"],
                   help="attention: the case6 block (headline); layer: attention + FF transformer layer")
    p.add_argument("--ff-dim", type=int, default=2560)
    p.add_argument("--layers", type=int, default=4, help="fsdp: number of dim x dim Dense layers")
    p.add_argument("--graph-steps", type=int, default=8,
                   help="training steps per captured HIP graph (the timed K steps replay K / G graphs of G "
                        "complete steps each: one graph launch per G steps; K %% G steps run one by one). "
                        "Every step still runs all its kernels - forward, backward, gradient all-reduce, "
                        "Adam - on the previous step's state; only the host launch is amortised")
    p.add_argument("--fp8", action="store_true", help="layer / ff: MX-fp8 FF GEMMs (CDNA4 block-scaled MFMA)")
    p.add_argument("--loss", default="sum", choices=["sum", "mse"],
                   help="sum: y.sum() as in case6_attention.py:211 (constant cotangent); mse: mean((y - target)^2) "
                        "against a synthetic target (a general, data-dependent cotangent)")
    p.add_argument("--rules", default="reference",
                   help="logical-axis rules preset (parallel/tensor.py PRESETS): reference (case6_attention.py:183-187), "
                        "case5 (embed->data: FSDP-sharded weights, case5_attention_dense.py:109-112), gspmd2d, megatron, dp")
    p.add_argument("--secondary", default=os.environ.get("LJS_BENCH_SECONDARY", "auto"),
                   choices=["auto", "on", "off", "0", "1"],
                   help="also time the reference's 2-D DP x TP layout ((N/2, 2) mesh) in the same job and report it "
                        "as the JSON line's 'secondary' object (auto: the headline block, --mesh dp, even N >= 2)")
    p.add_argument("--comm-timeout", type=float, default=None,
                   help="seconds a phase may run before the watchdog aborts the communicators and exits "
                        "(default LJS_COMM_TIMEOUT_S or 300)")
    a = p.parse_args()
    a.secondary = {"0": "off", "1": "on"}.get(a.secondary, a.secondary)
    return a


def _free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def _visible_gpu_count() -> int:
    """GPUs this job may use, counted WITHOUT initialising HIP in the launcher process: the KFD
    topology's GPU nodes (``gpu_id`` != 0), narrowed by ROCR/HIP/CUDA_VISIBLE_DEVICES.  Each rank
    re-checks its own device with torch before any GPU work (``_assert_rank_device``)."""
    import glob
    n = 0
    for f in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id"):
        try:
            with open(f) as fh:
                n += int(fh.read().strip() or "0") != 0
        except (OSError, ValueError):
            pass
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""])) if v.strip() else 0
    return n


def _launch_ranks(n: int) -> int:
    """Run this benchmark as n rank processes (one per GPU) and return their exit status.  This
    process never touches the GPU (no torch import): it counts devices from sysfs, starts
    ``torch.distributed.run`` as a CHILD (no exec) and forwards SIGTERM / SIGINT to it."""
    import signal
    import subprocess
    platform = os.environ.get("LJS_PLATFORM", "").lower()
    if platform != "cpu" and not os.environ.get("LJS_DIST_BACKEND"):
        have = _visible_gpu_count()
        if have < n:
            print(f"bench.py: --gpus {n} needs {n} visible GPUs, found {have} (KFD topology)", file=sys.stderr)
            return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    child = subprocess.Popen(cmd)

    def fwd(sig, _frame):
        try:
            child.send_signal(sig)
        except OSError:
            pass
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, fwd)
    return child.wait()


HEAD_DIMS_GPU = (64,)  # head dims the HIP attention kernels implement (ops/hip.py attention)


def check_args(args, on_gpu: bool) -> None:
    """Reject configurations the GPU path does not implement BEFORE any GPU work."""
    if on_gpu and args.model in ("attention", "layer") and args.dim_head not in HEAD_DIMS_GPU:
        raise SystemExit(f"bench.py: --dim-head {args.dim_head} is not supported by the HIP attention kernels "
                         f"(supported: {', '.join(map(str, HEAD_DIMS_GPU))})")
    if args.model == "fsdp" and args.mesh not in ("dp",) and not args.mesh.endswith("x1"):
        raise SystemExit("bench.py: --model fsdp shards weights over 'data' only; use --mesh dp or Nx1")
    if args.loss == "mse" and args.mode != "train":
        raise SystemExit("bench.py: --loss applies to --mode train")


def _assert_rank_device(world: int) -> None:
    """A GPU rank checks that its LOCAL_RANK names a visible device before using it."""
    import torch
    if os.environ.get("LJS_PLATFORM", "gpu").lower() == "cpu" or os.environ.get("LJS_DIST_BACKEND"):
        return
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    have = torch.cuda.device_count()
    if lr >= have:
        raise SystemExit(f"bench.py: rank {os.environ.get('RANK')} has LOCAL_RANK {lr} but only {have} GPUs are "
                         f"visible (world {world})")


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus is None:
        args.gpus = world
    if world == 1 and args.gpus > 1:
        sys.exit(_launch_ranks(args.gpus))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        os.environ.setdefault("LJS_PLATFORM", "gpu")
        os.environ.pop("LJS_NUM_DEVICES", None)
        _assert_rank_device(world)
    else:
        os.environ.setdefault("LJS_NUM_DEVICES", "1")
    import torch
    on_gpu = os.environ.get("LJS_PLATFORM", "").lower() != "cpu" and torch.cuda.is_available()
    check_args(args, on_gpu)
    import learning_jax_sharding_amd as ljs

    n = ljs.device_count()
    if world > 1:
        import torch.distributed as _dist
        assert _dist.is_initialized() and _dist.get_world_size() == world, "process group not initialised"
        assert n == world and ljs.local_device_count() == 1, (n, world)

    import torch.distributed as dist
    dist_on = dist.is_available() and dist.is_initialized()
    cuda = torch.cuda.is_available()
    rank = int(os.environ.get("RANK", "0"))
    # physical GPUs doing the work: one per rank, or the one GPU under N virtual devices
    n_gpus = world if world > 1 else (1 if cuda else 0)

    def barrier_sync():
        if cuda:
            torch.cuda.synchronize()
        if dist_on:
            dist.barrier()
        if cuda:
            torch.cuda.synchronize()

    # failure detection: a daemon thread polls every RCCL communicator's async error and each
    # phase's deadline; on an error or a hang it aborts the communicators, prints the phase and
    # the partitions, and exits non-zero (comm/watchdog.py) instead of hanging in a synchronize
    from learning_jax_sharding_amd.comm.backend import get_comm
    wd = get_comm().watchdog(args.comm_timeout) if dist_on else None

    def phase(name, timeout=None):
        if wd is not None:
            wd.phase(name, timeout)

    env = dict(n=n, world=world, torch=torch, ljs=ljs, dist=dist, dist_on=dist_on, cuda=cuda,
               barrier_sync=barrier_sync, phase=phase, probe=dist_on and world > 1)
    res = _measure_with_fallback(args, args.mesh, env)
    comm = "none"
    if dist_on:
        c = get_comm()
        comm = dist.get_backend() + ("+native-rccl" if getattr(c, "_native", None) is not None else "")
    rec = None
    detail = _comm_detail(env, res) if dist_on and world > 1 else None
    if rank == 0:
        rec = _record(args, res, n, n_gpus, cuda, comm)
        if detail is not None:
            rec["comm_detail"] = detail
    import threading
    print_lock, printed = threading.Lock(), []

    def print_once():
        # the main thread and the watchdog thread (on_fail) may both try: exactly one prints
        with print_lock:
            if rec is not None and not printed:
                printed.append(1)
                print(json.dumps(rec), flush=True)

    # the reference's own 2-D DP x TP layout (case6_attention.py:155-162,183-187; BASELINE config 4)
    # timed in the same job as a secondary result: the headline stays the DP layout
    if _want_secondary(args, n):
        def on_fail(reason):
            # a hang or RCCL error inside the secondary measurement: the headline, measured before
            # it, is still printed (with the error), and the job still exits with the watchdog's
            # non-zero code (None keeps comm/watchdog.EXIT_CODE): a run that hung never reads as a pass
            if rec is not None:
                rec["secondary"] = {"mesh": "2d", "error": reason[:300]}
            print_once()
            return None
        if wd is not None:
            wd.on_fail = on_fail
        try:
            env["probe"] = False
            if dist_on and hasattr(get_comm(), "routes"):
                get_comm().routes.clear()   # the secondary layout's routes are reported on their own
            res2 = _measure_with_fallback(args, "2d", env,
                                          phase_timeout=float(os.environ.get("LJS_BENCH_SECONDARY_TIMEOUT_S", "240")))
            # the 2-D layout's own collectives (gathers, all-to-alls): which path carried them
            # (collective: every rank)
            d2 = _comm_detail(env, res2) if dist_on and world > 1 else None
            if rec is not None:
                rec["secondary"] = {
                    "mesh": list(res2["mshape"]), "parallelism": _parallelism(args, res2["mshape"]),
                    "ms_per_step": round(res2["ms"], 4),
                    "tflops_per_gpu": round(res2["tflops_total"] / max(1, n_gpus if cuda else n), 3),
                    "value": round(res2["tflops_total"], 3), "comm": comm,
                    "graph_segments": res2["segs"], "steps_per_graph": res2["G"],
                    "warmup_steps_run": res2["warm_run"], "rules": args.rules,
                }
                if d2 is not None:
                    rec["secondary"]["comm_routes"] = d2["routes"]
                    rec["secondary"]["routes_agree_across_ranks"] = d2["routes_agree_across_ranks"]
                    rec["secondary"]["p2p_fallbacks"] = d2["p2p_fallbacks"]
        except Exception as e:   # (same on every rank: the measurement is SPMD)
            if rec is not None:
                rec["secondary"] = {"mesh": "2d", "error": f"{type(e).__name__}: {e}"[:300]}
        if wd is not None:
            wd.on_fail = None
    print_once()
    if dist_on:
        phase("shutdown")
        dist.barrier()
        if wd is not None:
            wd.stop()
        get_comm().close()          # ncclCommDestroy of the native communicators
        dist.destroy_process_group()


class _Remeasure(Exception):
    """A peer-memory collective failed at run time (a barrier timed out): every rank has moved to
    RCCL (comm/backend.DistComm.p2p_health) and the layout is measured again on it."""


def _p2p_check(env, where: str) -> None:
    if not env["dist_on"]:
        return
    from learning_jax_sharding_amd.comm.backend import get_comm
    c = get_comm()
    if hasattr(c, "p2p_health"):
        reason = c.p2p_health()     # collective: every rank checks here, all agree
        if reason is not None:
            raise _Remeasure(f"{where}: {reason}")


def _measure_with_fallback(args, mesh_arg, env, phase_timeout=None):
    """``_measure``, once more on RCCL if a peer-memory collective failed during it (the job is not
    aborted: the failure and the fallback are recorded in comm_detail.p2p_fallbacks)."""
    try:
        return _measure(args, mesh_arg, env, phase_timeout)
    except _Remeasure as e:
        print(f"bench.py: {e}; peer-memory collectives off, measuring again on RCCL", file=sys.stderr, flush=True)
        res = _measure(args, mesh_arg, env, phase_timeout)
        res["remeasured"] = str(e)[:300]
        return res


def _comm_detail(env, res):
    """Which collective path ran (every rank's view, checked for agreement), RCCL's own rank counts,
    the gradient buckets of the last backward, and the timed eager all-reduce of the gradient size
    through each path (``res['probe']``, measured before the timed region)."""
    from learning_jax_sharding_amd.comm.backend import get_comm
    from learning_jax_sharding_amd.parallel import data as _data
    dist = env["dist"]
    c = get_comm()
    det = c.comm_detail() if hasattr(c, "comm_detail") else {"backend": dist.get_backend()}
    mine = [(r["kind"], r["bytes"], r["path"]) for r in det.get("routes", [])]
    allr = [None] * dist.get_world_size()
    dist.all_gather_object(allr, mine)
    det["routes_agree_across_ranks"] = all(a == allr[0] for a in allr)
    det["grad_buckets"] = [{"bytes": b, "dtype": dt, "groups": [list(g) for g in gr]} for b, dt, gr in _data.LAST_BUCKETS]
    if res.get("probe") is not None:
        det["all_reduce_probe"] = res["probe"]
    if res.get("remeasured"):
        det["remeasured"] = res["remeasured"]
    return det


def _want_secondary(args, n) -> bool:
    """Time the reference's 2-D layout too: on by default for the headline block with an even
    device count >= 2 under the DP mesh (``--secondary off`` / LJS_BENCH_SECONDARY=0 disables)."""
    if args.secondary == "off":
        return False
    if args.secondary == "on":
        return n >= 2 and n % 2 == 0
    return args.model == "attention" and args.mesh == "dp" and n >= 2 and n % 2 == 0 and args.mode == "train"


def _mesh_shape(mesh_arg, n):
    if mesh_arg == "dp":
        return (n, 1)
    if mesh_arg == "2d":
        return (max(1, n // 2), 2 if n >= 2 else 1)
    return tuple(int(v) for v in mesh_arg.split("x"))


def _parallelism(args, mshape) -> str:
    par = f"dp{mshape[0]}" + (f"xtp{mshape[1]}" if mshape[1] > 1 else "")
    if args.model == "fsdp" or (args.rules in ("case5", "fsdp", "gspmd2d") and mshape[0] > 1):
        par = f"fsdp{mshape[0]}" + (f"xtp{mshape[1]}" if mshape[1] > 1 else "")
    return par


def _measure(args, mesh_arg, env, phase_timeout=None):
    """Build the model on the mesh ``mesh_arg``, capture, warm up and time ``args.steps`` steps
    (barrier + synchronize on both sides, max over ranks).  Returns the timing and its context."""
    torch, ljs, dist = env["torch"], env["ljs"], env["dist"]
    n, dist_on, cuda = env["n"], env["dist_on"], env["cuda"]
    if cuda:
        torch.cuda.reset_peak_memory_stats()
    barrier_sync, phase = env["barrier_sync"], env["phase"]
    from learning_jax_sharding_amd import nn, optim
    from learning_jax_sharding_amd.mesh import Mesh, create_device_mesh
    from learning_jax_sharding_amd.models import (DenseStack, MultiHeadAttention, TransformerLayer,
                                                  attention_block_flops, dense_stack_flops, feed_forward_flops,
                                                  transformer_layer_flops)
    from learning_jax_sharding_amd.parallel import fsdp
    from learning_jax_sharding_amd.sharding import NamedSharding, PartitionSpec as P
    from learning_jax_sharding_amd.training import TrainState

    mshape = _mesh_shape(mesh_arg, n)
    assert mshape[0] * mshape[1] == n, (mshape, n)
    mesh = Mesh(create_device_mesh(mshape), ("data", "model"))
    from learning_jax_sharding_amd.parallel.tensor import rules as _rules_preset
    rules = _rules_preset(args.rules)
    B = args.batch_per_gpu * n
    S, M = args.seq, args.dim
    if args.model == "layer":
        model = TransformerLayer(M, heads=args.heads, dim_head=args.dim_head, ff_dim=args.ff_dim, fp8=args.fp8)
    elif args.model == "ff":
        model = nn.FeedForward(args.ff_dim, fp8=args.fp8)
    elif args.model == "fsdp":
        model = DenseStack(M, layers=args.layers)
    else:
        model = MultiHeadAttention(M, heads=args.heads, dim_head=args.dim_head)
    x_sharding = NamedSharding(mesh, P("data", "model"))
    x = ljs.random.normal(ljs.random.PRNGKey(0), (B, S, M), sharding=x_sharding)

    def init_fn(k, x):
        params = model.init(k, x)["params"]
        return TrainState.create(apply_fn=model.apply, params=params, tx=optim.adam(1e-3))

    abstract = ljs.eval_shape(init_fn, ljs.random.PRNGKey(1), x)
    if args.model == "fsdp":
        # case3 at scale: every parameter (and its Adam moments) sharded over 'data'
        state_sharding = fsdp.fsdp_shardings(abstract, mesh, "data")
    else:
        state_sharding = nn.logical_to_mesh_sharding(nn.get_partition_spec(abstract), mesh, rules)
    state = ljs.jit(init_fn, out_shardings=state_sharding)(ljs.random.PRNGKey(1), x)

    target = None
    if args.loss == "mse":
        # a synthetic regression target shaped (and sharded) like the block's output
        target = ljs.random.normal(ljs.random.PRNGKey(2), (B, S, M), sharding=x_sharding)

    def train_step(state, x):
        def loss_fn(params):
            y = model.apply({"params": params}, x)
            if target is not None:
                return ljs.ops.core.mse_loss(y, target)
            return y.sum()
        grads = ljs.grad(loss_fn)(state.params)
        state = state.apply_gradients(grads=grads)
        if clock_probe:
            # diagnostics: the shader clock after every step (csrc/kernels/diag.hip; captured into
            # the graphs like the step's kernels, so every replayed step records one)
            from learning_jax_sharding_amd.ops import hip as _hip
            _hip.clock_probe(torch.device("cuda", torch.cuda.current_device()))
        return state

    def fwd_step(state, x):
        return model.apply({"params": state.params}, x)

    capture = not args.no_graph and torch.cuda.is_available()
    clock_probe = os.environ.get("LJS_CLOCK_PROBE") and torch.cuda.is_available()
    aten_trace = os.environ.get("LJS_ATEN_TRACE")   # diagnostics: eager steps, one traced (utils/aten_trace.py)
    if aten_trace:
        capture = False
    G = max(1, args.graph_steps) if (capture and args.mode == "train") else 1
    # the timed steps run through ONE captured graph: G becomes the largest divisor of the step
    # count not above --graph-steps (alternating the G-step and the 1-step graph made every switch
    # copy the whole train state into the other graph's static inputs inside the timed region:
    # --steps 20 with G = 8 ran 2-10 % slower than --steps 16)
    while G > 1 and args.steps % G:
        G -= 1
    if args.mode == "train":
        step = ljs.jit(train_step, in_shardings=(state_sharding, x_sharding), out_shardings=state_sharding,
                       donate_argnums=0, capture=capture)

        from learning_jax_sharding_amd.ops import linear as _lin

        def train_steps(state, x):  # G complete training steps, each on the previous one's state
            for i in range(G):
                # the next step's input is known: its bf16 cast runs in this step's optimizer
                # launch (or before a data-parallel gradient join; ops/linear.prefetch_next_input);
                # each step still casts its own input once, inside this graph
                if i + 1 < G:
                    _lin.prefetch_next_input(x)
                state = train_step(state, x)
            _lin.join_precasts()
            return state
        multi = ljs.jit(train_steps, in_shardings=(state_sharding, x_sharding), out_shardings=state_sharding,
                        donate_argnums=0, capture=capture) if G > 1 else None
    else:
        step = ljs.jit(fwd_step, in_shardings=(state_sharding, x_sharding), out_shardings=x_sharding,
                       capture=capture)
        multi = None

    def run(k):
        nonlocal state
        out = None
        if multi is not None:
            for _ in range(k // G):
                state = multi(state, x)
            k = k % G
        for _ in range(k):
            if args.mode == "train":
                state = step(state, x)
            else:
                out = step(state, x)
        return out

    with mesh, nn.axis_rules(rules):
        phase(f"capture + warmup ({mesh_arg})", phase_timeout)
        warm_run = 0   # every untimed step, capture steps included
        if multi is not None:
            # both graphs captured before the timed region, whatever W is
            run(2 * G)
            run(2)
            warm_run += 2 * G + 2
        run(max(1, args.warmup))
        warm_run += max(1, args.warmup)
        # untimed: at least --min-warmup steps in all (a fixed count, so every rank runs the
        # same collectives) - steps ~20-45 run under a measured clock dip (profiles/
        # r6b_clock_ramp.md) - ending in the G-step graph so the timed steps start in its buffers
        extra = max(0, args.min_warmup - warm_run)
        if multi is not None and extra % G:
            extra += G - extra % G   # whole G-step graphs: the timed steps start in its buffers
        if extra:
            run(extra)
            warm_run += extra
        # a peer-memory barrier that timed out during warmup: every rank moves to RCCL and this
        # layout is measured again (comm_detail.p2p_fallbacks records it)
        _p2p_check(env, f"warmup ({mesh_arg})")
        probe = None
        if env.get("probe"):
            from learning_jax_sharding_amd.parallel import data as _data
            gbytes = sum(b for b, _, _ in _data.LAST_BUCKETS)
            if gbytes:
                from learning_jax_sharding_amd.comm.probe import all_reduce_paths
                # (diagnostic only: a path that raises on every rank alike is reported, and the
                # measurement the record is for still runs)
                try:
                    probe = all_reduce_paths(gbytes)
                except Exception as e:  # noqa: BLE001
                    probe = [{"error": f"{type(e).__name__}: {e}"[:300]}]
        if aten_trace:
            from learning_jax_sharding_amd.utils.aten_trace import AtenTrace
            with AtenTrace(cuda_only=not os.environ.get("LJS_ATEN_TRACE_ALL"),
                           depth=int(os.environ.get("LJS_ATEN_TRACE_DEPTH", "6"))) as tr:
                run(1)
            if int(os.environ.get("RANK", "0")) == 0:
                tr.write(aten_trace)
        barrier_sync()
        phase(f"timed steps ({mesh_arg})", phase_timeout)
        t0 = time.perf_counter()
        run(args.steps)
        th = time.perf_counter()  # host side done enqueuing (diagnostic: host- vs device-bound)
        barrier_sync()
        t1 = time.perf_counter()
        phase(f"report ({mesh_arg})", phase_timeout)
        _p2p_check(env, f"timed steps ({mesh_arg})")
    elapsed = t1 - t0
    if clock_probe and int(os.environ.get("RANK", "0")) == 0:
        from learning_jax_sharding_amd.ops import hip as _hip
        recs = _hip.clock_probe_records(torch.device("cuda", torch.cuda.current_device()))
        with open(os.environ["LJS_CLOCK_PROBE"], "w") as f:
            json.dump({"warm_run": warm_run, "steps": args.steps, "records": recs}, f)
    if dist_on:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if cuda else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3
    segs = None
    if capture:
        caps = list((multi or step)._graphs.values())
        if caps:
            segs = sum(1 for it in caps[-1].graph.items if it[0] == "graph")
    if args.model == "ff":
        flops = feed_forward_flops(B, S, M, args.ff_dim, train=args.mode == "train")
    elif args.model == "fsdp":
        flops = dense_stack_flops(B, S, M, args.layers, train=args.mode == "train")
    elif args.model == "layer":
        flops = transformer_layer_flops(B, S, M, args.heads, args.dim_head, args.ff_dim, train=args.mode == "train")
    else:
        flops = attention_block_flops(B, S, M, args.heads, args.dim_head, train=args.mode == "train")
    # device memory held by this layout's graphs, state and caches (the G-step graph's private
    # pool grows with G: PERF_NOTES round 5, multi-step graphs)
    peak_gb = torch.cuda.max_memory_reserved() / 1e9 if cuda else None
    # free this layout's graphs and state before another layout is built (the secondary run)
    del state, step, multi
    return dict(ms=ms, tflops_total=flops / (ms * 1e-3) / 1e12, tokens_per_s=B * S / (ms * 1e-3),
                host_ms=(th - t0) / args.steps * 1e3, mshape=mshape, B=B, S=S, M=M, G=G, segs=segs,
                warm_run=warm_run, capture=capture, peak_gb=peak_gb, probe=probe)


def _record(args, res, n, n_gpus, cuda, comm):
    M, mshape = res["M"], res["mshape"]
    gemm = "MX-fp8" if args.fp8 else "bf16"
    model_desc = {
        "attention": f"case6 attention block (M={M}, heads={args.heads}x{args.dim_head}, bf16 compute, "
                     f"f32 params, Adam)",
        "layer": f"attention+FF transformer layer (M={M}, heads={args.heads}x{args.dim_head}, "
                 f"ff={args.ff_dim}, FF GEMMs {gemm}, f32 params, Adam)",
        "ff": f"case4 GSPMD feed-forward relu(x Win) Wout (M={M}, ff={args.ff_dim}, {gemm} GEMMs, "
              f"f32 params, Adam)",
        "fsdp": f"case3 fully-sharded matmul chain ({args.layers} x Dense {M}x{M}, relu, bf16 compute, "
                f"f32 params FSDP-sharded over data, Adam)",
    }[args.model]
    return {
        "metric": METRIC if args.model == "attention" else f"step-time ms + TFLOPS/GPU, {args.model} train step",
        "value": round(res["tflops_total"], 3),
        "unit": "TFLOPS, whole job (matmul FLOPs of fwd+bwd summed over the n_gpus GPUs; the per-GPU rate "
                "the metric names is tflops_per_gpu = value / n_gpus)",
        "n_gpus": n_gpus if cuda else n,
        "n_devices": n,
        "steps": args.steps,
        # the untimed steps actually run before the timed region: --warmup plus the clock-ramp
        # minimum (--min-warmup), so the field says what ran
        "warmup": res["warm_run"],
        "warmup_requested": args.warmup,
        "ms_per_step": round(res["ms"], 4),
        "tflops_per_gpu": round(res["tflops_total"] / max(1, n_gpus if cuda else n), 3),
        "tokens_per_s": round(res["tokens_per_s"], 1),
        "host_ms_per_step": round(res["host_ms"], 4),
        "peak_mem_reserved_gb": None if res["peak_gb"] is None else round(res["peak_gb"], 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": ("bf16+mx-fp8" if args.model == "layer" else "mx-fp8") if args.fp8 else "bf16",
        "data": "synthetic (random normal x, random-init weights)",
        "config": {"model": model_desc,
                   "global_batch": res["B"], "seq_len": res["S"], "parallelism": _parallelism(args, mshape),
                   "mode": args.mode, "hip_graph": res["capture"], "graph_segments": res["segs"],
                   "steps_per_graph": res["G"], "warmup_steps_run": res["warm_run"], "mesh": list(mshape),
                   "comm": comm, "grad_wire": os.environ.get("LJS_GRAD_COMM_DTYPE", "fp32"),
                   "loss": "y.sum()" if args.loss == "sum" else "mean((y - target)^2)", "rules": args.rules},
    }


if __name__ == "__main__":
    main()
