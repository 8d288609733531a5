#!/usr/bin/env python3
"""Fast-SCNN MI355X benchmark — BASELINE.json metric:
    "images/sec fwd+bwd @1024x2048 bs=8 per GPU; 1/2/4/8-GPU scaling"

Workload (BASELINE.json configs[2] / [3]): one training step = forward + cross-entropy +
backward + fused SGD (lr 0.01, momentum 0.9, wd 1e-4) of Fast-SCNN (19 classes) on a synthetic
Cityscapes-shaped batch of 8 x 3 x 1024 x 2048 per GPU, bf16 activations with fp32 master
weights and fp32 statistics.  Weights come from the portable generator (random init, PyTorch
default law), inputs/targets from the same generator with rank-dependent seeds (5 % ignore).
N > 1: one process per GPU (torchrun), gradients all-reduced over RCCL in four buckets
overlapped with the staged backward; weak scaling (8 images per GPU).

    python bench.py [--gpus N --steps K --warmup W]

Rank 0 prints ONE JSON line.  Extra objects: roofline of the dominant kernel family (kernel time
per launch from the committed rocprofv3 summary of this command, beside the live HIP-event time
of its dispatches in the timed region; algorithmic bytes per SURVEY.md §8(d)),
cpu_baseline (the oracle restatement timed on this host's cores on a bounded sample), and the
forward-only fp32 inference rate (cfg2) for the north-star forward target.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec fwd+bwd @1024x2048 bs=8 per GPU; 1/2/4/8-GPU scaling"
HBM_PEAK_GBS = 8000.0
MFMA_PEAK_TFS = {"bf16": 2500.0, "fp32": 157.3}
# launch-profiler kinds (csrc/common.hpp ProfKind); each launcher accounts the algorithmic bytes /
# flops of SURVEY.md §8(d) for its launch shape (csrc/*.hip ProfScope), DESIGN.md §3
PROF_KINDS = {1: "conv0_fwd", 2: "dw_fwd", 3: "dw_dgrad", 4: "dw_wgrad", 5: "gemm_nt",
              6: "gemm_tn", 7: "bn_apply", 8: "bn_bwd_apply", 9: "upsample", 11: "ce_head",
              12: "conv0_wgrad", 13: "bn_bwd_reduce", 14: "bn_finalize", 15: "ppm_branches"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one process per GPU); default: WORLD_SIZE or 1")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--width", type=int, default=2048)
    ap.add_argument("--classes", type=int, default=19)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--profile-kind", type=int, default=0, help="0 = dominant (census)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-forward", action="store_true")
    ap.add_argument("--unfused-loss", action="store_true",
                    help="materialise full-res logits and run the separate CE kernels")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (0: this process's CPU share)")
    ap.add_argument("--no-cfg5", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the fp16 train-step line and the published-configuration line")
    return ap.parse_args()


def launch_ranks(n):
    """--gpus N > 1 without a launcher: start N ranks (one process per GPU) through
    torch.distributed.run as a CHILD process, before this process touches the GPU, and exit
    with its status (train.py:170-171's DataParallel over N devices becomes N processes)."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd, env=env)


def cpu_share():
    """Threads this process may use: its CPU affinity, capped by OMP_NUM_THREADS when set."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def prof(lib, kind, fn, max_launches, per_launch=False):
    """Kernel time (ms), launches, algorithmic bytes and flops of one kernel family over fn();
    per_launch: also [(layer, us, bytes, flops)] in issue order."""
    import torch
    from fast_scnn_pytorch_amd import _lib
    _lib.check(lib.fscnn_prof_begin(kind, max_launches), "fscnn_prof_begin")
    fn()
    torch.cuda.synchronize()
    ms, n, b, f = (ctypes.c_double(), ctypes.c_longlong(), ctypes.c_double(), ctypes.c_double())
    _lib.check(lib.fscnn_prof_end(ctypes.byref(ms), ctypes.byref(n), ctypes.byref(b),
                                  ctypes.byref(f)), "fscnn_prof_end")
    if not per_launch:
        return ms.value, n.value, b.value, f.value
    recs = []
    for i in range(n.value):
        k, t, by, fl, tag = (ctypes.c_int(), ctypes.c_float(), ctypes.c_double(), ctypes.c_double(),
                             ctypes.c_char_p())
        _lib.check(lib.fscnn_prof_launch(i, ctypes.byref(k), ctypes.byref(t), ctypes.byref(by),
                                         ctypes.byref(fl), ctypes.byref(tag)), "fscnn_prof_launch")
        recs.append((tag.value.decode(), t.value * 1e3, by.value, fl.value))
    return ms.value, n.value, b.value, f.value, recs


def family_report(recs, peak_gbs):
    """Per-family HBM fraction from kernel time, and each launch's layer / us / fraction."""
    us = sum(r[1] for r in recs)
    by = sum(r[2] for r in recs)
    gbs = by / (us * 1e-6) / 1e9 if us > 0 else 0.0
    return {"launches": len(recs), "us": round(us, 1), "GBps": round(gbs, 1),
            "hbm_frac": round(gbs / peak_gbs, 4),
            "layers": [[r[0], round(r[1], 1), round(r[2] / (r[1] * 1e-6) / 1e9 / peak_gbs, 3)
                        if r[1] > 0 else 0.0] for r in recs]}


def cpu_baseline(args):
    """Oracle restatement (port) timed on this host's cores on bounded samples: the train step
    (the metric's unit, at cfg3's own 8 x 3 x 1024 x 2048), the cfg2 forward (8 x 3 x 1024 x 2048,
    eval) beside forward_fp32, the cfg1 forward (1 x 3 x 768 x 768, the demo.py path) and the cfg5
    forward (32 x 3 x 480 x 640, 2 classes; fp32 — the CPU has no fp16 arithmetic path)."""
    import numpy as np
    import torch
    from fast_scnn_pytorch_amd import arch, portable_init
    from oracle import fast_scnn_ref as ref  # checker / CPU baseline only
    threads = args.cpu_threads or cpu_share()
    torch.set_num_threads(threads)
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in
          arch.portable_state_dict(args.classes, seed=0).items()}

    def timed(fn, reps, budget):
        fn()
        times = []
        t_end = time.perf_counter() + budget
        while len(times) < reps and (not times or time.perf_counter() < t_end):
            t0 = time.perf_counter()
            fn()
            times.append(time.perf_counter() - t0)
        return sorted(times)[len(times) // 2], len(times)

    out = {}
    with torch.no_grad():
        x8 = torch.from_numpy(portable_init.input_tensor(1, (8, 3, args.height, args.width)))
        med, n = timed(lambda: ref.forward(sd, x8, args.classes), 3, 12.0)
        out["forward_cfg2"] = {"value": round(8 / med, 3), "unit": "images/s",
                               "ms_per_batch": round(1e3 * med, 1),
                               "sample": "eval fp32 8x3x%dx%d, median of %d after 1 warm-up"
                                         % (args.height, args.width, n)}
        del x8
        x1 = torch.from_numpy(portable_init.input_tensor(1, (1, 3, 768, 768)))
        med, n = timed(lambda: ref.forward(sd, x1, args.classes), 10, 5.0)
        out["forward_cfg1"] = {"value": round(1 / med, 3), "unit": "images/s",
                               "ms_per_image": round(1e3 * med, 2),
                               "sample": "eval fp32 1x3x768x768 (demo.py path), median of %d" % n}
        del x1
        sd5 = {k: torch.from_numpy(np.asarray(v)) for k, v in
               arch.portable_state_dict(2, seed=0).items()}
        x5 = torch.from_numpy(portable_init.input_tensor(1, (32, 3, 480, 640)))
        med, n = timed(lambda: ref.forward(sd5, x5, 2), 3, 6.0)
        out["forward_cfg5"] = {"value": round(32 / med, 3), "unit": "images/s",
                               "ms_per_batch": round(1e3 * med, 1),
                               "sample": "eval fp32 32x3x480x640, 2 classes, median of %d after "
                                         "1 warm-up" % n}
        del x5, sd5
    nb = args.batch
    for k, v in sd.items():
        if v.is_floating_point() and "running" not in k:
            v.requires_grad_(True)
    x = torch.from_numpy(portable_init.input_tensor(1, (nb, 3, args.height, args.width)))
    t = torch.from_numpy(portable_init.target_tensor(3, (nb, args.height, args.width),
                                                     args.classes, 0.05))

    def step():
        for v in sd.values():
            v.grad = None
        outs, _, _ = ref.forward(sd, x, args.classes, training=True, dropout_seed=5)
        ref.cross_entropy(outs[0], t).backward()

    med, n = timed(step, 2, 20.0)
    res = {"value": round(nb / med, 4), "unit": "images/s", "cores": threads, "kind": "port",
           "sample": "oracle/fast_scnn_ref.py train step (fwd+CE+bwd, fp32) on %d x 3 x %d x %d, "
                     "median of %d after 1 warm-up, torch CPU %d threads"
                     % (nb, args.height, args.width, n, threads),
           "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
           "torch": torch.__version__}
    res.update(out)
    return res


def _timed_steps(step, n, warm):
    import torch
    for _ in range(warm):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def train_fp16_rate(args, model, x, t, dev):
    """cfg3's step (fused CE head, FusedSGD, 8 x 3 x 1024 x 2048, 19 classes) in the reference's
    own AMP arithmetic: train.py:269's autocast() (fp16 activations and weight copies, fp32
    master weights / statistics / accumulation) over fp32 images."""
    import torch
    from fast_scnn_pytorch_amd.optim import FusedSGD
    opt = FusedSGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    xf = x.float()

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda"):
            loss = model.forward_loss(xf, t)
        loss.backward()
        opt.step()
    n = max(5, args.steps // 2)
    sec = _timed_steps(step, n, 3)
    return {"value": round(args.batch / sec, 2), "unit": "images/s", "ms_per_step": round(1e3 * sec, 3),
            "dtype": "fp16", "steps": n,
            "config": "cfg3 train step under torch.autocast('cuda') (fp16, train.py:269), fp32 images"}


def published_config_rate(args, dev):
    """The reference's only published training number (PERFORMANCE_MONITORING.md:24-25,57-66:
    232.9 samples/s) is for its train.py loop at: TuSimple (2 classes), batch 8, 768 x 768 crops
    (train.py:48 --crop-size default), fp16 AMP with GradScaler (train.py:200-201,268-275), aux
    head (aux_weight 0.4, train.py:55), MixDiceLoss (train.py:70,183-184), SGD momentum 0.9 /
    wd 1e-4.  The same loop here, including its per-iteration loss.item() (train.py:283) and
    GradScaler's inf check; synthetic images already on the device (the reference's timer also
    covers the batch's host-to-device copy and the data wait is excluded)."""
    import numpy as np
    import torch
    from fast_scnn_pytorch_amd import arch, portable_init
    from fast_scnn_pytorch_amd.loss import MixDiceLoss
    from fast_scnn_pytorch_amd.optim import FusedSGD
    from models.fast_scnn import FastSCNN
    m = FastSCNN(2, aux=True)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in
                       arch.portable_state_dict(2, aux=True, seed=0).items()})
    m = m.to(dev).train()
    B, S = 8, 768
    xi = torch.from_numpy(portable_init.input_tensor(7, (B, 3, S, S))).to(dev)
    ti = torch.from_numpy(portable_init.target_tensor(8, (B, S, S), 2, 0.0)).to(dev)
    crit = MixDiceLoss(aux=True, aux_weight=0.4)
    opt = FusedSGD(m.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    scaler = torch.amp.GradScaler("cuda")
    losses = []

    def step():
        opt.zero_grad()
        with torch.autocast("cuda"):
            outputs = m(xi)
            loss = crit(outputs, ti)
        scaler.scale(loss).backward()
        scaler.step(opt)
        scaler.update()
        losses.append(loss.item())
    n = max(10, args.steps)
    sec = _timed_steps(step, n, 5)
    val = B / sec
    return {"value": round(val, 2), "unit": "samples/s", "ms_per_step": round(1e3 * sec, 3),
            "steps": n, "published": 232.9, "vs_published": round(val / 232.9, 2),
            "published_source": "PERFORMANCE_MONITORING.md:24-25,57-66 (GPU not stated)",
            "dtype": "fp16", "loss_first_last": [round(losses[0], 4), round(losses[-1], 4)],
            "config": "train.py loop: TuSimple 2 classes, bs 8, 768x768, autocast fp16 + "
                      "GradScaler, aux=True (0.4), MixDiceLoss, SGD m 0.9 wd 1e-4, "
                      "loss.item() per step"}


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus is not None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if env_world is not None and args.gpus is not None and int(env_world) != args.gpus:
        sys.exit("bench.py: --gpus %d but WORLD_SIZE=%s" % (args.gpus, env_world))
    import torch
    import torch.distributed as dist
    import _fscnn_boot
    _fscnn_boot.load()
    import numpy as np
    from fast_scnn_pytorch_amd import _lib, arch, portable_init
    from fast_scnn_pytorch_amd.loss import cross_entropy
    from fast_scnn_pytorch_amd.optim import FusedSGD
    from models.fast_scnn import FastSCNN

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local if world > 1 else 0)
    lib = _lib.load()
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32

    model = FastSCNN(args.classes)
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in
          arch.portable_state_dict(args.classes, seed=0).items()}
    model.load_state_dict(sd)
    model = model.to(dev).train()
    net = model
    if world > 1:
        from fast_scnn_pytorch_amd.ddp import DistributedFastSCNN
        net = DistributedFastSCNN(model)
    opt = FusedSGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    B, H, W = args.batch, args.height, args.width
    x = torch.from_numpy(portable_init.input_tensor(1 + rank, (B, 3, H, W))).to(dev).to(dt)
    t = torch.from_numpy(portable_init.target_tensor(3 + rank, (B, H, W), args.classes,
                                                     0.05)).to(dev)

    def step():
        opt.zero_grad(set_to_none=True)
        if args.unfused_loss:
            loss = cross_entropy(net(x)[0], t)
        else:
            # same loss and gradients as cross_entropy(net(x)[0], t) (tests/test_gpu_model.py
            # test_fused_loss_head_*), evaluated at 1/8 resolution without full-res logits
            loss = net.forward_loss(x, t)
        loss.backward()
        opt.step()
        return loss

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        loss = step()
    barrier()
    first_loss = float(loss.item())

    # census (untimed): which kernel family dominates the step
    kind = args.profile_kind
    census = {}
    if kind == 0:
        for k, name in PROF_KINDS.items():
            ms, n, b, f = prof(lib, k, step, 4096)
            census[name] = round(ms, 4)
        kind = max(PROF_KINDS, key=lambda k: census[PROF_KINDS[k]])
    barrier()

    # ---- timed region: K steps; the dominant family's dispatches in the last tenth of the timed
    # steps carry kernel-bound HIP events (hipExtLaunchKernelGGL: each event pair holds its
    # dispatch's own start / end timestamps, the kernel time rocprofv3 reports; no marker
    # packets on the stream); the events are created before the region
    nprof = max(1, args.steps // 10)
    _lib.check(lib.fscnn_prof_begin(kind, 512 * nprof), "fscnn_prof_begin")
    ms, n, b, f = (ctypes.c_double(), ctypes.c_longlong(), ctypes.c_double(), ctypes.c_double())
    _lib.check(lib.fscnn_prof_end(ctypes.byref(ms), ctypes.byref(n), ctypes.byref(b),
                                  ctypes.byref(f)), "fscnn_prof_end")
    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i == args.steps - nprof:
            lib.fscnn_prof_begin(kind, 512 * nprof)
            if world > 1:
                net.timing = True  # per-bucket all-reduce / exposed comm events (ddp.py)
        loss = step()
    barrier()
    elapsed = time.perf_counter() - t0
    _lib.check(lib.fscnn_prof_end(ctypes.byref(ms), ctypes.byref(n), ctypes.byref(b),
                                  ctypes.byref(f)), "fscnn_prof_end")
    last_loss = float(loss.item())
    per_rank_ms = [round(1e3 * elapsed / args.steps, 3)]
    if world > 1:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        allt = [torch.zeros_like(tt) for _ in range(world)]
        dist.all_gather(allt, tt)
        per_rank_ms = [round(1e3 * float(v.item()) / args.steps, 3) for v in allt]
        elapsed = max(float(v.item()) for v in allt)

    # per-step distribution (BASELINE.md §2 asks for a median over >= 20 iterations): K more
    # steps AFTER the timed region, each bracketed by events on the caller's stream (one event per
    # step boundary; it idles the stream ~7 us, so these steps are not the ones `value` times)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(max(20, args.steps) + 1)]
    evs[0].record()
    for i in range(1, len(evs)):
        step()
        evs[i].record()
    torch.cuda.synchronize()
    step_ms = sorted(evs[i - 1].elapsed_time(evs[i]) for i in range(1, len(evs)))
    median_ms = step_ms[len(step_ms) // 2]
    # pointwise (1x1 conv) MFMA utilisation, one profiled step per family (untimed): the
    # forward / dgrad GEMMs (gemm_nt) and the weight gradients (gemm_tn), dense bf16 peak
    mfma_util = {}
    for pk, pname in ((5, "gemm_nt"), (6, "gemm_tn")):
        pms, pn, pb, pf = prof(lib, pk, step, 4096)
        if pms > 0:
            tfs = pf / (pms * 1e-3) / 1e12
            mfma_util[pname] = {"launches": pn, "ms": round(pms, 4), "tflops": round(tfs, 2),
                                "peak_tflops": MFMA_PEAK_TFS[args.dtype],
                                "frac": round(tfs / MFMA_PEAK_TFS[args.dtype], 4)}
    # the train step's depthwise families (forward, input gradient, weight gradient) from kernel
    # time, each launch named by its layer (north_star's depthwise >= 60 % of HBM target)
    depthwise = {}
    for pk, pname in ((2, "dw_fwd"), (3, "dw_dgrad"), (4, "dw_wgrad")):
        res = prof(lib, pk, step, 4096, per_launch=True)
        depthwise[pname] = family_report(res[4], HBM_PEAK_GBS)
        depthwise[pname]["_recs"] = res[4]
    barrier()

    value = world * B * args.steps / elapsed
    avg_ms = ms.value / max(1, n.value)
    bytes_per_launch = b.value / max(1, n.value)
    flops_per_launch = f.value / max(1, n.value)
    ach_gbs = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    ach_tfs = flops_per_launch / (avg_ms * 1e-3) / 1e12 if avg_ms > 0 else 0.0
    mfma_peak = MFMA_PEAK_TFS[args.dtype]
    kname = PROF_KINDS.get(kind, str(kind))
    # depthwise families from kernel time: algorithmic bytes per step (live) over the family's
    # rocprofv3 kernel time per step
    try:
        fams = json.load(open(os.path.join(ROOT, "profiles", "rocprof_family_%s.json" % args.dtype)))
        for pname, rep_ in depthwise.items():
            fk = fams["families"].get(pname)
            if fk and fk.get("ms_per_step"):
                by = sum(l_[2] for l_ in rep_.pop("_recs", []))
                rep_["kernel_time_frac"] = round(by / (fk["ms_per_step"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                rep_["kernel_ms_per_step"] = fk["ms_per_step"]
    except Exception:
        pass
    for rep_ in depthwise.values():
        rep_.pop("_recs", None)
    # the headline: the family's KERNEL time from the committed rocprofv3 --kernel-trace --stats
    # summary of this bench command (profiles/rocprof_family_<dtype>.json, regenerated with each
    # round's measurement set: tools/gpu_measure.sh, tools/rocprof_family.py), so `frac` is what
    # profiles/ reproduces; the live HIP-event figure of this run (each event pair also spans the
    # launch gap before its kernel) is the `event` sub-object
    rpf = os.path.join(ROOT, "profiles", "rocprof_family_%s.json" % args.dtype)
    k_us, k_src = None, None
    if os.path.exists(rpf):
        try:
            fam = json.load(open(rpf))
            fk = fam["families"].get(kname)
            if fk and fk.get("avg_us"):
                k_us = fk["avg_us"]
                k_src = "profiles/%s (round %s)" % (os.path.basename(rpf), fam.get("round", "?"))
        except Exception:
            pass
    use_us = k_us if k_us else avg_ms * 1e3
    k_gbs = bytes_per_launch / (use_us * 1e-6) / 1e9 if use_us > 0 else 0.0
    k_tfs = flops_per_launch / (use_us * 1e-6) / 1e12 if use_us > 0 else 0.0
    if kname in ("gemm_nt", "gemm_tn") and k_tfs / mfma_peak > k_gbs / HBM_PEAK_GBS:
        roof = {"bound": "mfma", "achieved": round(k_tfs, 3), "peak": mfma_peak,
                "unit": "TFLOP/s", "frac": round(k_tfs / mfma_peak, 4)}
    else:
        roof = {"bound": "hbm", "achieved": round(k_gbs, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(k_gbs / HBM_PEAK_GBS, 4)}
    roof.update({"kernel": kname, "launches": n.value, "avg_launch_us": round(use_us, 2),
                 "algo_bytes_per_launch": round(bytes_per_launch),
                 "algo_flops_per_launch": round(flops_per_launch), "traffic": None})
    roof["timing"] = (("kernel time per launch from %s (rocprofv3 --kernel-trace --stats of this "
                       "bench command)" % k_src) if k_us else
                      "HIP events bound to each dispatch (no committed rocprofv3 summary found)")
    roof["event"] = {"avg_launch_us": round(avg_ms * 1e3, 2), "achieved": round(ach_gbs, 1),
                     "frac": round(ach_gbs / HBM_PEAK_GBS, 4),
                     "timing": "this run, live: HIP events bound to each dispatch of the family "
                               "(hipExtLaunchKernelGGL) over the last tenth of the timed steps; "
                               "each pair also spans the launch gap before its kernel"}
    # HBM traffic per launch from the PMC counters of a committed profiling run (rocprofv3 --pmc
    # cannot run inside this process); labelled with its file and round
    pmc = os.path.join(ROOT, "profiles", "pmc_%s_%s.json" % (kname, args.dtype))
    if os.path.exists(pmc):
        try:
            pj = json.load(open(pmc))
            roof["traffic"] = pj.get("hbm_bytes_per_launch")
            roof["traffic_source"] = "profiles/%s (PMC FETCH_SIZE+WRITE_SIZE, round %s)" % (
                os.path.basename(pmc), pj.get("round", pj.get("tag", "?")))
        except Exception:
            pass

    result = {
        "metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True,
        "step_ms_distribution": {"median": round(median_ms, 3), "min": round(step_ms[0], 3),
                                 "max": round(step_ms[-1], 3), "n": len(step_ms),
                                 "timing": "HIP events per step boundary on the caller's stream, "
                                           "%d steps after the timed region (rank 0)" % len(step_ms)},
        "mfma_utilisation": dict(mfma_util, note="1x1-conv GEMM families, kernel time over one "
                                 "profiled step each; algorithmic flops 2*M*N*K per launch"),
        "depthwise_train": dict(depthwise, note="cfg3 train step, one profiled step per family, "
                                "HIP events bound to each dispatch (each spans its launch gap); "
                                "layers: [module, us, HBM fraction]; kernel_time_frac: the "
                                "family's algorithmic bytes per step over its rocprofv3 kernel "
                                "time per step (profiles/rocprof_family_<dtype>.json); dw_wgrad "
                                "runs on the low-priority side stream beside the main stream"),
        "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
        "data": "synthetic (portable counter-based generator; random-init weights, default law)",
        "config": {"workload": ("cfg3 train step: fwd + CE(ignore -1) + bwd + fused SGD" + (" (unfused CE)" if args.unfused_loss else " (fused low-res upsample+CE head)")),
                   "model": "FastSCNN (19 classes)", "global_batch": world * B,
                   "per_gpu_batch": B, "resolution": [H, W], "parallelism": "dp%d" % world},
        "roofline": roof,
        "loss": {"after_warmup": round(first_loss, 5), "final": round(last_loss, 5)},
        "per_rank_ms_per_step": per_rank_ms,
        "comm": {"backend": dist.get_backend() if world > 1 else None,
                 "world_size": dist.get_world_size() if world > 1 else 1,
                 "buckets": 4 if world > 1 else 0},
    }
    if world > 1:
        net.timing = False
        cs = net.comm_stats()
        if cs:
            # HIP events on the comm stream around each bucket's all-reduce (bucket order: head,
            # bottleneck3, bottleneck2, bottleneck1+LTD) and the comm time left after the
            # backward's last kernel, over the last tenth of the timed steps (rank 0's view)
            result["comm"].update(cs)
            result["comm"]["bucket_mb"] = [round(4 * (e - b) / 1e6, 3)
                                           for b, e in model.native().stage_ranges]
    if census:
        result["kernel_ms_per_step_census"] = census
        result["census_note"] = ("time per family over one profiled step each (HIP events bound "
                                 "to the dispatches, each spanning its launch gap); the families "
                                 "overlap on two streams, so the sum is not a breakdown of "
                                 "ms_per_step")

    # forward-only inference (rank 0, N=1 only): cfg2 fp32 (north-star forward target), cfg1
    # (demo.py: 1 x 3 x 768 x 768, latency) and cfg5 (TuSimple 32 x 3 x 480 x 640, C=2)
    if rank == 0 and world == 1 and not args.no_forward:
        model.eval()
        x32 = x.float()

        def fwd_rate(m, xin, nrep):
            with torch.no_grad():
                for _ in range(3):
                    m(xin)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                for _ in range(nrep):
                    m(xin)
                torch.cuda.synchronize()
            return (time.perf_counter() - t1) / nrep

        fe = fwd_rate(model, x32, max(5, args.steps // 2))
        # the fused inference blocks' matrix work (algorithmic flops of expand / depthwise /
        # project, conv0 / pointwise, dw / pw) per kernel time, against the fp32 matrix spec and
        # against the ceiling of the six-product split-bf16 form they run (2.5 PF / 6)
        fused = {}
        with torch.no_grad():
            for pk, pname in ((16, "ir_block"), (18, "dsconv"), (17, "ltd_stem")):
                fms, fn, fb, ff = prof(lib, pk, lambda: model(x32), 256)
                if fms > 0:
                    tfs = ff / (fms * 1e-3) / 1e12
                    fused[pname] = {"launches": fn, "us": round(fms * 1e3, 1),
                                    "tflops": round(tfs, 1),
                                    "frac_fp32_matrix": round(tfs / MFMA_PEAK_TFS["fp32"], 3),
                                    "frac_split_bf16": round(tfs / (MFMA_PEAK_TFS["bf16"] / 6), 3)}
        result["forward_fp32"] = {"value": round(B / fe, 2), "unit": "images/s",
                                  "ms_per_batch": round(1e3 * fe, 3),
                                  "config": "cfg2 eval fp32 %dx3x%dx%d" % (B, H, W),
                                  "fused_blocks_mfma": fused}
        x1 = torch.from_numpy(portable_init.input_tensor(1, (1, 3, 768, 768))).to(dev)
        f1 = fwd_rate(model, x1, 20)
        result["forward_cfg1"] = {"value": round(1 / f1, 2), "unit": "images/s",
                                  "ms_per_image": round(1e3 * f1, 3),
                                  "config": "cfg1 eval fp32 1x3x768x768 (demo.py path)"}
        del x1
        if not args.no_cfg5:
            m5 = FastSCNN(2)
            m5.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in
                                arch.portable_state_dict(2, seed=0).items()})
            m5 = m5.to(dev).eval()
            # fp16 images in, fp16 MFMA arithmetic (fp32 accumulation), fp16 logits out
            x5 = torch.from_numpy(portable_init.input_tensor(1, (32, 3, 480, 640))).to(dev).half()
            f5 = fwd_rate(m5, x5, 10)
            result["forward_cfg5"] = {"value": round(32 / f5, 2), "unit": "images/s",
                                      "ms_per_batch": round(1e3 * f5, 3),
                                      "dtype": "fp16",
                                      "config": "cfg5 eval 32x3x480x640, 2 classes"}
            del m5, x5
        model.train()

    if rank == 0 and world == 1 and not args.no_extra:
        result["train_fp16"] = train_fp16_rate(args, model, x, t, dev)
        result["train_published_cfg"] = published_config_rate(args, dev)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args)

    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
