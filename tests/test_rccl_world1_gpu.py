"""Every collective the DP path issues under RCCL ("nccl"), on a real RCCL communicator.

RCCL refuses two ranks on one GPU ("Duplicate GPU detected"), so the multi-rank logic is covered by
the gloo tests (test_dp*.py, test_zero*.py) and the 8-GPU runs are the driver's. What one GPU can
prove is that this ROCm / RCCL build accepts each call exactly as the nccl branches issue it —
op, dtype, async handle, in-place device buffer — so an N > 1 run does not die on the first bucket:

* grad_sync.py:103-111 / 185-187   all_reduce AVG, async, fp32 bucket
* grad_sync.py:400-404             reduce_scatter_tensor AVG, async, fp32 (ZeRO gradients)
* grad_sync.py:587                 all_gather_into_tensor, bf16 (ZeRO weights)
* grad_sync.py:202                 broadcast of device tensors (sync_module_states)
* grad_sync.py:567, trainer_step.py:93 / 131   all_reduce SUM / MAX / MIN, fp32 / fp64 scalars
* seqlen_balancing.py:117          all_reduce MAX, int64 (micro-batch count)
* dp_algos.py:65, protocol.py:558  all_gather of device tensors (group statistics, batches)
* grad_sync.py:171                 barrier

Run in a child process (its own communicator, torn down before the test returns)."""

import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

_CHILD = textwrap.dedent(
    """
    import os, torch, torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{os.environ['PORT']}", rank=0,
                            world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    g = torch.Generator(device=dev).manual_seed(0)
    buf = torch.randn(1 << 22, device=dev, generator=g)
    want = buf.clone()
    dist.all_reduce(buf, op=dist.ReduceOp.AVG, async_op=True).wait()
    assert torch.equal(buf, want), "all_reduce AVG"
    out = torch.empty_like(buf)
    dist.reduce_scatter_tensor(out, buf, op=dist.ReduceOp.AVG, async_op=True).wait()
    assert torch.equal(out, want), "reduce_scatter_tensor AVG"
    w = torch.empty(1 << 20, dtype=torch.bfloat16, device=dev)
    mine = want[: 1 << 20].to(torch.bfloat16)
    dist.all_gather_into_tensor(w, mine)
    assert torch.equal(w, mine), "all_gather_into_tensor bf16"
    for dt in (torch.float32, torch.bfloat16):
        t = want[:4096].to(dt)
        b = t.clone()
        dist.broadcast(b, src=0)
        assert torch.equal(b, t), f"broadcast {dt}"
    for dt in (torch.float32, torch.float64, torch.int64):
        for op in (dist.ReduceOp.SUM, dist.ReduceOp.MAX, dist.ReduceOp.MIN):
            t = (want[:8] * 100).to(dt)
            r = t.clone()
            dist.all_reduce(r, op=op)
            assert torch.equal(r, t), f"all_reduce {op} {dt}"
    for dt in (torch.float32, torch.float64, torch.int64, torch.bool):
        t = (want[:1000] > 0).to(dt) if dt == torch.bool else (want[:1000] * 7).to(dt)
        parts = [torch.empty_like(t)]
        dist.all_gather(parts, t)
        assert torch.equal(parts[0], t), f"all_gather {dt}"
    objs = [None]
    dist.all_gather_object(objs, {"uid": ["a", "b"]})
    assert objs[0] == {"uid": ["a", "b"]}
    dist.barrier()
    torch.cuda.synchronize()
    dist.destroy_process_group()
    print("rccl world-1 collectives ok", flush=True)
    """
)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_rccl_accepts_every_dp_collective():
    env = dict(os.environ, PORT=str(_free_port()), MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-c", _CHILD], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    assert "rccl world-1 collectives ok" in r.stdout
