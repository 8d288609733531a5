"""Is the training step GPU-bound?  Times the bench step (bench.py's step(): zero_grad,
forward_loss, backward, FusedSGD.step) three ways: host enqueue time per step (no sync),
wall time per step (synchronised), and the host time of each phase.

    python tools/host_overhead.py [--steps 30] [--batch 8 --height 1024 --width 2048]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--width", type=int, default=2048)
    ap.add_argument("--classes", type=int, default=19)
    args = ap.parse_args()
    import numpy as np
    import torch
    import _fscnn_boot
    _fscnn_boot.load()
    from fast_scnn_pytorch_amd import arch, portable_init
    from fast_scnn_pytorch_amd.optim import FusedSGD
    from models.fast_scnn import FastSCNN

    dev = torch.device("cuda", 0)
    model = FastSCNN(args.classes)
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in
          arch.portable_state_dict(args.classes, seed=0).items()}
    model.load_state_dict(sd)
    model = model.to(dev).train()
    opt = FusedSGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=1e-4)
    B, H, W = args.batch, args.height, args.width
    x = torch.from_numpy(portable_init.input_tensor(1, (B, 3, H, W))).to(dev).to(torch.bfloat16)
    t = torch.from_numpy(portable_init.target_tensor(3, (B, H, W), args.classes, 0.05)).to(dev)
    phase = {"zero_grad": 0.0, "forward_loss": 0.0, "backward": 0.0, "opt.step": 0.0}

    def step(timed=False):
        t0 = time.perf_counter()
        opt.zero_grad(set_to_none=True)
        t1 = time.perf_counter()
        loss = model.forward_loss(x, t)
        t2 = time.perf_counter()
        loss.backward()
        t3 = time.perf_counter()
        opt.step()
        t4 = time.perf_counter()
        if timed:
            phase["zero_grad"] += t1 - t0
            phase["forward_loss"] += t2 - t1
            phase["backward"] += t3 - t2
            phase["opt.step"] += t4 - t3
        return loss

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    K = args.steps
    # (1) host enqueue rate with a deep queue
    t0 = time.perf_counter()
    for _ in range(K):
        step(timed=True)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    # (2) GPU time per step between step-start events
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
    for i in range(K):
        ev[i].record()
        step()
    ev[K].record()
    torch.cuda.synchronize()
    gpu = [ev[i].elapsed_time(ev[i + 1]) for i in range(K)]
    # (3) one step at a time, synchronised: GPU latency of an isolated step
    iso = []
    for _ in range(10):
        torch.cuda.synchronize()
        s0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        iso.append(time.perf_counter() - s0)
    # (4) host cost of one step with an empty launch queue (no back-pressure), and a profile
    import cProfile
    import pstats
    enq = []
    prof = cProfile.Profile()
    for i in range(10):
        torch.cuda.synchronize()
        s0 = time.perf_counter()
        if i >= 5:
            prof.enable()
        step()
        if i >= 5:
            prof.disable()
        enq.append(time.perf_counter() - s0)
    torch.cuda.synchronize()
    print("host enqueue of one step, empty queue: median %.3f ms" % (1e3 * sorted(enq)[5]))
    st = pstats.Stats(prof)
    st.sort_stats("tottime").print_stats(18)
    print("host enqueue  %.3f ms/step   wall %.3f ms/step" % (1e3 * t_enq / K, 1e3 * t_all / K))
    print("event-to-event GPU step  median %.3f ms  min %.3f  max %.3f"
          % (sorted(gpu)[K // 2], min(gpu), max(gpu)))
    print("isolated step (sync)  median %.3f ms" % (1e3 * sorted(iso)[5]))
    for k, v in phase.items():
        print("  host %-13s %.3f ms/step" % (k, 1e3 * v / K))


if __name__ == "__main__":
    main()
