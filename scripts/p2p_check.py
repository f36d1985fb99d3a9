"""Multi-process check of the IPC peer-memory collectives (comm/p2p.py, ``ipc`` mode).

Launched by tests/test_p2p_gpu.py under torch.distributed.run with the gloo backend; the
ranks share the box's single MI355X, which exercises every piece of the N-GPU path (IPC
export/import of the uncached staging buffers, the cross-process flag barrier, the one- and
two-shot kernels, DistComm routing) except the xGMI transport itself.
"""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from learning_jax_sharding_amd.comm import p2p  # noqa: E402


def inputs(n, numel, dtype, seed):
    out = []
    for r in range(n):
        g = torch.Generator().manual_seed(seed * 100 + r)
        out.append(torch.randn(numel, generator=g).to(dtype))
    return out


def main():
    dist.init_process_group("gloo")
    rank, n = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    grp = p2p.P2PGroup([dev] * n, 2 << 20, rank=rank, pg=dist.group.WORLD)

    for seed, (numel, dtype) in enumerate([(1024, torch.float32), (50 * 1024, torch.bfloat16),
                                           (256 * 1024, torch.float32), (96, torch.bfloat16)]):
        xs = inputs(n, numel, dtype, seed)
        mine = xs[rank].to(dev)
        # all-reduce: f32 accumulation in member order == the local oracle, bitwise
        ref = xs[0].float()
        for r in range(1, n):
            ref = ref + xs[r].float()
        out = grp.all_reduce({rank: mine})[rank]
        assert torch.equal(out.cpu(), ref.to(dtype)), ("all_reduce", numel, dtype)
        # all-gather
        ag = grp.all_gather({rank: mine})[rank]
        assert torch.equal(ag.cpu(), torch.stack(xs)), ("all_gather", numel)
        if numel % (8 * n) == 0:
            # reduce-scatter of [n, chunk] and all-to-all
            chunk = numel // n
            rs = grp.reduce_scatter({rank: mine.view(n, chunk)})[rank]
            assert torch.equal(rs.cpu(), ref.to(dtype).view(n, chunk)[rank]), ("reduce_scatter", numel)
            a2a = grp.all_to_all({rank: mine.view(n, chunk)})[rank]
            want = torch.stack([xs[r].view(n, chunk)[rank] for r in range(n)])
            assert torch.equal(a2a.cpu(), want), ("all_to_all", numel)
    grp.check_error()

    # the framework route: DistComm sends small collectives through the p2p group
    os.environ["LJS_P2P"] = "1"
    os.environ.setdefault("LJS_PLATFORM", "gpu")
    from learning_jax_sharding_amd.comm.backend import DistComm
    from learning_jax_sharding_amd.runtime.devices import initialize_distributed
    initialize_distributed()
    comm = DistComm()
    x = torch.full((64, 32), float(rank + 1), device=dev)
    y = comm.all_reduce({comm.me: x}, [tuple(range(n))])[comm.me]
    assert torch.all(y == n * (n + 1) / 2), y
    assert comm._p2p_groups, "DistComm did not take the p2p path"
    # ... and, once built, the route is capturable (no graph cut at this collective)
    assert comm.graph_safe("all_reduce", x, [tuple(range(n))]), "p2p all-reduce not graph-safe"
    assert not comm.graph_safe("all_reduce", torch.empty(4 << 20, device=dev), [tuple(range(n))]) or \
        comm._native is not None

    # HIP-graph capture of the ipc collectives: replays keep advancing the device-side barrier
    # counter, so captured members stay in step; results follow the (re-filled) static input
    xin = torch.zeros(4096, device=dev)
    xg = torch.zeros(2 * 1024, dtype=torch.bfloat16, device=dev)
    grp.all_reduce({rank: xin})
    torch.cuda.synchronize()
    dist.barrier()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        yout = grp.all_reduce({rank: xin})[rank]
        gout = grp.all_gather({rank: xg})[rank]
    torch.cuda.synchronize()
    dist.barrier()
    for it in range(3):
        xin.fill_(float(rank + 1 + it))
        xg.fill_(float(rank - it))
        graph.replay()
        torch.cuda.synchronize()
        want = float(sum(r + 1 + it for r in range(n)))
        assert torch.all(yout == want), (it, yout[:4])
        for r in range(n):
            assert torch.all(gout[r] == float(r - it)), (it, r)
    grp.check_error()
    dist.barrier()

    # same-group collectives issued alternately on the compute stream and a side stream (a weight
    # prefetch next to the activation gathers): the group orders each after the previous one, so
    # the one staging buffer and the barrier sequence are never shared by two in flight - eager and
    # inside one capture
    side = torch.cuda.Stream(device=dev)
    ins = [torch.full((8192,), float(rank + 10 * j), device=dev) for j in range(6)]

    def alternate():
        outs = []
        for j, t in enumerate(ins):
            if j % 2:
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):
                    outs.append(grp.all_gather({rank: t})[rank])
                # (no join here: the next compute-stream collective is ordered by the group)
            else:
                outs.append(grp.all_gather({rank: t})[rank])
        torch.cuda.current_stream(dev).wait_stream(side)
        return outs

    def check_alt(outs):
        for j, o in enumerate(outs):
            for r in range(n):
                assert torch.all(o[r] == float(r + 10 * j)), ("two-stream all_gather", j, r)

    check_alt(alternate())
    torch.cuda.synchronize()
    dist.barrier()
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g2):
        alt_out = alternate()
    torch.cuda.synchronize()
    dist.barrier()
    for _ in range(2):
        g2.replay()
        torch.cuda.synchronize()
        check_alt(alt_out)
    grp.check_error()
    dist.barrier()

    # failure detection: a barrier nobody else joins times out into the error word, no hang
    dist.barrier()
    if rank == 0:
        os.environ["LJS_P2P_TIMEOUT_MS"] = "300"
        grp._barrier()
        try:
            grp.check_error()
            raise AssertionError("lone barrier did not time out")
        except RuntimeError as e:
            assert "timed out" in str(e)
    dist.barrier()
    torch.cuda.synchronize()
    dist.barrier()
    grp.close()
    for g in comm._p2p_groups.values():
        g.close()
    print(f"P2P OK rank {rank}", flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
