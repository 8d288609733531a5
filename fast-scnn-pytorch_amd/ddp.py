"""Data parallelism for the HIP Fast-SCNN: one process per GPU, gradient all-reduce over RCCL.

Replaces ``torch.nn.DataParallel(model, device_ids=[0, 1, 2])`` (train.py:170-171), which
replicated parameters, scattered the batch and gathered full-resolution logits to cuda:0 every
step.  Here every rank owns its own shard of the batch and computes its loss locally; the only
exchange is the gradient all-reduce.  The native backward runs in four stages (head / bottleneck3
/ bottleneck2 / bottleneck1+LTD, the buckets of SURVEY.md §8(e)); as soon as a stage has been
enqueued its contiguous slice of the flat gradient arena is all-reduced asynchronously (on a
communication stream on the GPU), overlapping the remaining backward (depthwise and GEMM)
kernels; the last stage waits for every bucket.

BatchNorm statistics stay per rank (no SyncBN), like DataParallel's per-replica statistics;
running statistics are those of each rank (rank 0's are the ones to checkpoint).

``timing = True`` records, per step, each bucket's all-reduce time (HIP events on the
communication stream around the collective) and the exposed communication time (from the end of
the backward's last kernel on the compute stream to the end of the last all-reduce);
``comm_stats()`` averages them over the recorded steps.
"""
import collections

import torch
import torch.distributed as dist


class DistributedFastSCNN(torch.nn.Module):
    def __init__(self, model, process_group=None, broadcast=True):
        super().__init__()
        if not dist.is_initialized():
            raise RuntimeError("torch.distributed must be initialised (one process per GPU)")
        self.module = model
        self.pg = process_group
        self.world = dist.get_world_size(process_group)
        self.backend = dist.get_backend(process_group)
        self.comm_stream = torch.cuda.Stream() if self._on_gpu() else None
        self._works = []
        self.timing = False
        self._step_events = []   # per recorded step: ([(stage, start, end)], main_end)
        self._cur_events = []
        # (stage, begin, end, async) of the all-reduces issued, the last 64 (4 per step)
        self.bucket_log = collections.deque(maxlen=64)
        if broadcast:
            self.broadcast_parameters()
        model.grad_stage_hook = self._stage_hook

    def _on_gpu(self):
        return next(self.module.parameters()).is_cuda

    @torch.no_grad()
    def broadcast_parameters(self):
        """Make every rank start from rank 0's parameters and buffers (one call per arena)."""
        if self._on_gpu():
            ar = self.module.arena()
            for t in (ar["P"], ar["R"], ar["NBT"]):
                dist.broadcast(t, 0, group=self.pg)
        else:
            for t in list(self.module.parameters()) + list(self.module.buffers()):
                dist.broadcast(t.data, 0, group=self.pg)

    def _stage_hook(self, stage, G, begin, end):
        bucket = G[begin:end]
        self.bucket_log.append((stage, begin, end, True))
        if self.comm_stream is None:  # CPU tensors (gloo): asynchronous, waited at the last stage
            self._works.append(self._reduce(bucket, async_op=True))
            if stage == 3:
                self._finish()
            return
        cur = torch.cuda.current_stream()
        self.comm_stream.wait_stream(cur)
        with torch.cuda.stream(self.comm_stream):
            t0 = self._event() if self.timing else None
            wp = self._reduce(bucket, async_op=True)
            if self.timing:
                # the comm stream waits for the collective's own stream, so the next event
                # completes when this bucket's all-reduce has
                if wp is not None and wp[0] is not None:
                    wp[0].wait()
                self._cur_events.append((stage, t0, self._event()))
            self._works.append(wp)
        if stage == 3:
            main_end = self._event(cur) if self.timing else None
            self._finish()
            cur.wait_stream(self.comm_stream)
            if self.timing:
                self._step_events.append((self._cur_events, main_end))
            self._cur_events = []

    @staticmethod
    def _event(stream=None):
        e = torch.cuda.Event(enable_timing=True)
        e.record(stream)
        return e

    def _finish(self):
        for wp in self._works:
            if wp is None:
                continue
            work, post = wp
            if work is not None:
                work.wait()
            if post is not None:
                post()
        self._works = []

    def _reduce(self, bucket, async_op=False):
        """Average ``bucket`` over the ranks: (work, post) — post runs after the work completes
        (gloo has no AVG: SUM, then the division)."""
        if self.world == 1:
            return None
        if self.backend == "nccl":
            return dist.all_reduce(bucket, op=dist.ReduceOp.AVG, group=self.pg,
                                   async_op=async_op), None
        w = dist.all_reduce(bucket, op=dist.ReduceOp.SUM, group=self.pg, async_op=async_op)
        post = lambda: bucket.div_(self.world)  # noqa: E731
        if not async_op:
            post()
            return w, None
        return w, post

    def comm_stats(self, reset=True):
        """Mean per-bucket all-reduce ms (stage order: head, bottleneck3, bottleneck2,
        bottleneck1+LTD), mean exposed ms and the recorded step count (synchronises)."""
        if not self._step_events:
            return None
        torch.cuda.synchronize()
        per = {}
        exposed = []
        for evs, main_end in self._step_events:
            for stage, a, b in evs:
                per.setdefault(stage, []).append(a.elapsed_time(b))
            if evs and main_end is not None:
                exposed.append(max(0.0, main_end.elapsed_time(evs[-1][2])))
        out = {"bucket_allreduce_ms": [round(sum(v) / len(v), 4) for _, v in sorted(per.items())],
               "exposed_ms": round(sum(exposed) / max(1, len(exposed)), 4),
               "steps": len(self._step_events)}
        if reset:
            self._step_events = []
        return out

    def allreduce_grads(self):
        """Explicit gradient averaging for models that do not run the native staged backward."""
        for p in self.module.parameters():
            if p.grad is not None:
                self._reduce(p.grad)

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def forward_loss(self, x, target, ignore_index=-1):
        """Fused forward + CE of the local shard; backward all-reduces gradients per stage."""
        return self.module.forward_loss(x, target, ignore_index=ignore_index)
