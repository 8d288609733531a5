"""Data-parallel layer (ddp.py) on CPU with gloo, world_size 2.

The HIP backward itself needs a GPU; here the staged gradient hook is driven with per-rank
gradient arenas exactly as ``FastSCNN._run_backward`` calls it (stage s, flat arena G, the
executor's [begin, end) range for that stage), which is the whole data-path exchange of a step
(replacing ``nn.DataParallel``'s reduce-add, train.py:170-171).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2  # spawned ranks inherit sys.path (repo root from conftest.py)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, port, q):
    try:
        import _fscnn_boot
        _fscnn_boot.load()
        from fast_scnn_pytorch_amd.ddp import DistributedFastSCNN
        from models.fast_scnn import FastSCNN
        torch.manual_seed(100 + rank)  # different init per rank before the broadcast
        dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d" % port, rank=rank,
                                world_size=WORLD)
        m = FastSCNN(19)
        with torch.no_grad():
            m.classifier.conv[1].bias.fill_(float(rank + 1))
            m.learning_to_downsample.conv.conv[1].running_mean.fill_(float(rank + 3))
        ddp = DistributedFastSCNN(m)
        res = {}
        res["bias"] = m.classifier.conv[1].bias.clone()
        res["rmean"] = m.learning_to_downsample.conv.conv[1].running_mean.clone()
        res["w0"] = m.learning_to_downsample.conv.conv[0].weight.clone()

        nat = m.native()
        G = torch.arange(nat.p_total, dtype=torch.float32) * (rank + 1) + 10.0 * rank
        calls = []
        for s in range(4):
            b, e = nat.stage_ranges[s]
            calls.append((s, b, e))
            m.grad_stage_hook(s, G, b, e)
        res["G"] = G
        res["ranges"] = calls
        res["log"] = list(ddp.bucket_log)
        res["pending"] = len(ddp._works)
        res["world"] = ddp.world

        # explicit path (allreduce_grads) on ordinary .grad tensors
        for p in m.parameters():
            p.grad = torch.full_like(p, float(rank))
        ddp.allreduce_grads()
        res["grad_mean"] = float(next(m.parameters()).grad.mean())
        dist.barrier()
        dist.destroy_process_group()
        # plain numpy copies: torch tensors would travel as shared memory owned by this process
        q.put((rank, {k: (v.detach().numpy() if torch.is_tensor(v) else v) for k, v in res.items()}))
    except Exception as exc:  # pragma: no cover - surfaced by the parent
        q.put((rank, repr(exc)))


@pytest.fixture(scope="module")
def results():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(WORLD):
        rank, res = q.get(timeout=240)
        out[rank] = res
    for p in procs:
        p.join(timeout=60)
    for r, res in out.items():
        assert not isinstance(res, str), "rank %d failed: %s" % (r, res)
        for k, v in list(res.items()):
            if hasattr(v, "dtype") and not isinstance(v, (int, float)):
                res[k] = torch.from_numpy(v)
    return out


def test_broadcast_from_rank0(results):
    r0, r1 = results[0], results[1]
    assert torch.equal(r0["bias"], r1["bias"]) and float(r0["bias"][0]) == 1.0
    assert torch.equal(r0["rmean"], r1["rmean"]) and float(r0["rmean"][0]) == 3.0
    assert torch.equal(r0["w0"], r1["w0"])


def test_stage_buckets_average_gradients(results):
    r0, r1 = results[0], results[1]
    assert r0["world"] == WORLD
    n = r0["G"].numel()
    idx = torch.arange(n, dtype=torch.float32)
    expect = (idx * 1 + 0.0 + idx * 2 + 10.0) / 2
    covered = torch.zeros(n, dtype=torch.bool)
    for _, b, e in r0["ranges"]:
        covered[b:e] = True
    # every element inside a stage bucket is the rank average; both ranks agree bit-exactly
    assert torch.equal(r0["G"], r1["G"])
    assert torch.allclose(r0["G"][covered], expect[covered])


def test_bucket_to_stage_mapping_async(results):
    """Every stage issues exactly its own bucket as an asynchronous all-reduce (async_op=True,
    waited at the last stage: nothing is pending after the backward), in backward order."""
    for r in (0, 1):
        log = results[r]["log"]
        assert [(s, b, e) for s, b, e, _ in log] == [tuple(c) for c in results[r]["ranges"]]
        assert all(a for *_, a in log)
        assert results[r]["pending"] == 0


def test_stage_ranges_partition_all_parameters(results):
    import _fscnn_boot
    _fscnn_boot.load()
    from models.fast_scnn import FastSCNN
    m = FastSCNN(19)
    nat = m.native()
    ranges = [r[1:] for r in results[0]["ranges"]]
    # stages run head → LTD, i.e. descending arena order, disjoint and gap-free over params
    for (b0, e0), (b1, e1) in zip(ranges, ranges[1:]):
        assert b1 < e1 <= b0 < e0
    owner = {}
    for name, off, numel in nat.params:
        hits = [s for s, (b, e) in enumerate(ranges) if b <= off and off + numel <= e]
        assert len(hits) == 1, name
        owner[name] = hits[0]
    assert owner["classifier.conv.1.weight"] == 0
    assert owner["global_feature_extractor.ppm.out.conv.0.weight"] == 0
    assert owner["global_feature_extractor.bottleneck3.0.block.2.weight"] == 1
    assert owner["global_feature_extractor.bottleneck2.0.block.0.conv.0.weight"] == 2
    assert owner["learning_to_downsample.conv.conv.0.weight"] == 3
    sizes = {s: sum(n for name, _, n in nat.params if owner[name] == s) for s in range(4)}
    # SURVEY.md §8(e) bucket sizes
    assert sizes == {0: 114963, 1: 550464, 2: 303168, 3: 169456}


def test_allreduce_grads_explicit(results):
    assert results[0]["grad_mean"] == pytest.approx(0.5)
    assert results[1]["grad_mean"] == pytest.approx(0.5)
