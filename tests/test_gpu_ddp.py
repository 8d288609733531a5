"""Data parallelism through the REAL staged HIP backward (replaces train.py:170-171's DataParallel):
two ranks on the one GPU of the box (gloo over CUDA tensors — the RCCL path is the same hook with
backend "nccl"), each running DistributedFastSCNN.forward_loss + backward on its own shard.  The
per-stage bucket all-reduce of the flat gradient arena must give exactly the mean of the two
single-process gradient arenas, on every rank, and one FusedSGD step keeps the replicas identical.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, port, q):
    try:
        import torch.distributed as dist
        import _fscnn_boot
        _fscnn_boot.load()
        from fast_scnn_pytorch_amd import arch, portable_init
        from fast_scnn_pytorch_amd.ddp import DistributedFastSCNN
        from fast_scnn_pytorch_amd.optim import FusedSGD
        from models.fast_scnn import FastSCNN
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                                world_size=WORLD)
        sd = {k: torch.from_numpy(np.asarray(v)) for k, v in
              arch.portable_state_dict(19, seed=0).items()}
        shape = (2, 3, 96, 160)
        xs = [torch.from_numpy(portable_init.input_tensor(10 + r, shape)).to(dev)
              for r in range(WORLD)]
        ts = [torch.from_numpy(portable_init.target_tensor(20 + r, (2, 96, 160), 19, 0.05)).to(dev)
              for r in range(WORLD)]

        def fresh():
            m = FastSCNN(19)
            m.load_state_dict(sd)
            m = m.to(dev).train()
            m._dropout_seed = 7
            return m

        # single-process gradient arenas of both shards (no hook)
        local = []
        for r in range(WORLD):
            m = fresh()
            m.forward_loss(xs[r], ts[r]).backward()
            local.append(torch.cat([p.grad.flatten() for p in m.parameters()]).cpu())
            del m
        # the data-parallel step on this rank's shard
        m = fresh()
        ddp = DistributedFastSCNN(m)
        loss = ddp.forward_loss(xs[rank], ts[rank])
        loss.backward()
        torch.cuda.synchronize()
        avg = torch.cat([p.grad.flatten() for p in m.parameters()]).cpu()
        opt = FusedSGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
        opt.step()
        torch.cuda.synchronize()
        params = torch.cat([p.detach().flatten() for p in m.parameters()]).cpu()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, {"local0": local[0].numpy(), "local1": local[1].numpy(),
                      "avg": avg.numpy(), "params": params.numpy(), "loss": float(loss.item())}))
    except Exception as exc:  # pragma: no cover - surfaced by the parent
        import traceback
        q.put((rank, traceback.format_exc() + repr(exc)))


@pytest.fixture(scope="module")
def results():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    env_ipc = os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    assert env_ipc == "0"
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(WORLD):
            rank, res = q.get(timeout=100)
            out[rank] = res
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r, res in out.items():
        assert not isinstance(res, str), "rank %d failed: %s" % (r, res)
    return out


def test_staged_allreduce_is_the_mean_of_the_shard_gradients(results):
    r0, r1 = results[0], results[1]
    # both ranks computed the same single-process arenas (deterministic kernels)
    assert np.array_equal(r0["local0"], r1["local0"]) and np.array_equal(r0["local1"], r1["local1"])
    want = (r0["local0"] + r0["local1"]) / np.float32(2)  # gloo: fp32 sum, then / world
    assert np.array_equal(r0["avg"], want)
    assert np.array_equal(r1["avg"], want)


def test_replicas_stay_identical_after_the_step(results):
    assert np.array_equal(results[0]["params"], results[1]["params"])
    assert results[0]["loss"] != results[1]["loss"]  # different shards
