"""The reference's own multi-GPU call of the module: ``torch.nn.DataParallel(model, device_ids)``
(train.py:170-171; SURVEY.md §8(b) "Threading / streams").

DataParallel replicates the module every step (``replicate``: shallow ``__dict__`` copies whose
parameters are broadcast, non-leaf tensors), runs the replicas concurrently from one worker
thread per device (``parallel_apply``) and reduce-adds their gradients onto the source module's
parameters.  The box has one GPU, so the replicas here share cuda:0 — two threads driving the
native executor at once, on the same plan, side stream and events — which is the harder case for
thread safety.  Replica 0 aliases the module's arenas; replica 1 holds broadcast copies (packed
into its own arenas per call).

Gate: the reduce-added gradients equal the mean of the two single-thread shard steps (fp32: bit
for bit up to the fp32 sum of the two halves; bf16: same), the running statistics follow
replica 0 (DataParallel semantics), and eval outputs of each replica equal the single-module
outputs.
"""
import numpy as np
import pytest
import torch
from torch.nn.parallel import gather, parallel_apply, replicate

from fast_scnn_pytorch_amd import arch, portable_init
from fast_scnn_pytorch_amd.loss import cross_entropy
from models.fast_scnn import FastSCNN

pytestmark = pytest.mark.gpu

SHAPE = (2, 3, 96, 160)


def _sd():
    return {k: torch.from_numpy(np.asarray(v)) for k, v in
            arch.portable_state_dict(19, seed=0, variant="bnrand").items()}


def _fresh(dev, train=True):
    m = FastSCNN(19)
    m.load_state_dict(_sd())
    m = m.to(dev)
    m.train(train)
    m._dropout_seed = 11
    return m


def _shards(dev, dtype=torch.float32):
    xs = [torch.from_numpy(portable_init.input_tensor(30 + r, SHAPE)).to(dev).to(dtype)
          for r in range(2)]
    ts = [torch.from_numpy(portable_init.target_tensor(40 + r, (SHAPE[0],) + SHAPE[2:], 19,
                                                       0.05)).to(dev) for r in range(2)]
    return xs, ts


def _grads(m):
    return {n: p.grad.detach().float().clone() for n, p in m.named_parameters()}


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_replicate_parallel_apply_matches_single_thread_shards(dtype):
    dev = torch.device("cuda", 0)
    xs, ts = _shards(dev, dtype)
    # single-thread reference: each shard on its own fresh module, loss halved like the mean
    ref, ref_bn = [], []
    for r in range(2):
        m = _fresh(dev)
        (cross_entropy(m(xs[r])[0], ts[r]) * 0.5).backward()
        ref.append(_grads(m))
        ref_bn.append({k: v.detach().clone() for k, v in m.state_dict().items()
                       if "running" in k or "num_batches" in k})
    torch.cuda.synchronize()

    model = _fresh(dev)
    for step in range(2):  # a second step re-replicates from the (unchanged) module
        model.zero_grad(set_to_none=True)
        reps = replicate(model, [0, 0])
        outs = parallel_apply(reps, [(xs[0],), (xs[1],)], devices=[0, 0])
        loss = sum(cross_entropy(o[0], t) for o, t in zip(outs, ts)) * 0.5
        loss.backward()
        torch.cuda.synchronize()
        worst = 0.0
        for n, p in model.named_parameters():
            exp = ref[0][n] + ref[1][n]
            got = p.grad.detach().float()
            d = (got - exp).abs().max().item()
            scale = exp.abs().max().item() + 1e-30
            worst = max(worst, d / scale)
            assert d <= 1e-6 * scale, "%s (step %d): max|d| %g (scale %g)" % (n, step, d, scale)
        print("dtype %s step %d: worst relative grad difference %.3g" % (dtype, step, worst))
    # running statistics follow replica 0 (shard 0), updated twice from the same start
    m0 = _fresh(dev)
    for _ in range(2):
        m0(xs[0])
    sd_dp, sd_0 = model.state_dict(), m0.state_dict()
    for k in ref_bn[0]:
        assert torch.equal(sd_dp[k], sd_0[k]), k


def test_replica_eval_outputs_and_dataparallel_module():
    dev = torch.device("cuda", 0)
    xs, _ = _shards(dev)
    model = _fresh(dev, train=False)
    with torch.no_grad():
        single = [model(x)[0].clone() for x in xs]
        reps = replicate(model, [0, 0], detach=True)
        outs = parallel_apply(reps, [(xs[0],), (xs[1],)], devices=[0, 0])
        both = gather(outs, 0)[0]
    torch.cuda.synchronize()
    assert torch.equal(both, torch.cat(single, 0))
    # eval.py-style call without no_grad (eval mode: no autograd graph is recorded)
    out = replicate(model, [0, 0])[1](xs[1])[0]
    assert torch.equal(out, single[1])
    # train.py:170-171 on this box: DataParallel over the one device (plain module call)
    dp = torch.nn.DataParallel(model, device_ids=[0]).cuda()
    with torch.no_grad():
        assert torch.equal(dp(xs[0])[0], single[0])


def test_replica_on_copied_arena_writes_back_running_stats():
    """A replica that does not alias the module (broadcast copies) updates its own buffers."""
    dev = torch.device("cuda", 0)
    xs, _ = _shards(dev)
    model = _fresh(dev)
    rep = replicate(model, [0, 0])[1]
    before = model.state_dict()["learning_to_downsample.conv.conv.1.running_mean"].clone()
    rep(xs[0])
    torch.cuda.synchronize()
    m0 = _fresh(dev)
    m0(xs[0])
    rb = rep.learning_to_downsample.conv.conv[1].running_mean
    assert torch.equal(rb, m0.learning_to_downsample.conv.conv[1].running_mean)
    assert int(rep.learning_to_downsample.conv.conv[1].num_batches_tracked) == 1
    # the module itself is untouched by replica 1 (DataParallel keeps replica 0's statistics)
    assert torch.equal(model.state_dict()["learning_to_downsample.conv.conv.1.running_mean"],
                       before)


def test_model_on_non_current_device():
    """A model on cuda:k called while another device is current (``--device cuda:1`` with
    cuda:0 current): every native call runs under a guard of the input's device, and the
    executor's weight-gradient side stream is bound to the caller's stream device (skipped, one
    stream, if they ever differ).  Gradients equal the same step run with its device current.
    Needs >= 2 GPUs (skipped on the one-GPU box)."""
    n = torch.cuda.device_count()
    if n < 2:
        pytest.skip("needs two GPUs")
    dev = torch.device("cuda", n - 1)
    xs, ts = _shards(dev)
    with torch.cuda.device(dev):
        m = _fresh(dev)
        cross_entropy(m(xs[0])[0], ts[0]).backward()
        ref = _grads(m)
    torch.cuda.set_device(0)
    m = _fresh(dev)
    cross_entropy(m(xs[0])[0], ts[0]).backward()
    torch.cuda.synchronize(dev)
    for k, v in _grads(m).items():
        assert torch.equal(v, ref[k]), k
