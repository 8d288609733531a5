"""Fast-SCNN with the reference interface, executed by the gfx950 HIP library.

Drop-in for ``models/fast_scnn.py`` of Shinokawa/Fast-SCNN-pytorch:

* ``__all__ = ['FastSCNN', 'get_fast_scnn']`` (reference :13);
* ``FastSCNN(num_classes, aux=False, **kwargs)`` (:16-17) with the same submodule tree, so
  ``state_dict()`` keys / shapes (Appendix A of SURVEY.md) and attribute paths such as
  ``model.classifier.conv[1].out_channels`` or ``ppm.conv1.conv[0]`` are unchanged;
* ``forward(x)`` returns a ``tuple`` of NCHW logits at the input resolution (:33-46);
* ``get_fast_scnn(dataset, pretrained, root, map_cpu, **kwargs)`` (:240-256) with a static
  NUM_CLASS table instead of importing the data loaders (no torchvision dependency).

The parameters are re-homed into one flat fp32 arena (64-B aligned tensors, layout owned by the
C++ executor), running statistics into a second arena; ``.grad`` tensors returned by backward
are views of one flat gradient arena, so the fused SGD and the RCCL all-reduce each touch a
single buffer.  The submodules are parameter containers only: the whole network runs as one
native forward and one staged native backward.  CPU tensors raise — there is no fallback.
"""
import os
import threading

import torch
import torch.nn as nn

from . import _lib
from .arch import NUM_CLASS

__all__ = ["FastSCNN", "get_fast_scnn"]


# ---------------------------------------------------------------------------------------------
# parameter containers (attribute schema of models/fast_scnn.py:49-237)
# ---------------------------------------------------------------------------------------------
class _Container(nn.Module):
    def forward(self, *args, **kwargs):  # pragma: no cover - guard
        raise RuntimeError("%s is a parameter container; call the FastSCNN module"
                           % type(self).__name__)


def _seq_conv_bn_relu(cin, cout, k, stride, padding, groups=1):
    return nn.Sequential(nn.Conv2d(cin, cout, k, stride, padding, groups=groups, bias=False),
                         nn.BatchNorm2d(cout), nn.ReLU(True))


class _ConvBNReLU(_Container):
    """models/fast_scnn.py:49-61 (padding defaults to 0)."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=0, **kwargs):
        super().__init__()
        self.conv = _seq_conv_bn_relu(in_channels, out_channels, kernel_size, stride, padding)


class _DSConv(_Container):
    """models/fast_scnn.py:64-79: dw3x3 → BN → ReLU → pw → BN → ReLU."""

    def __init__(self, dw_channels, out_channels, stride=1, **kwargs):
        super().__init__()
        dw = _seq_conv_bn_relu(dw_channels, dw_channels, 3, stride, 1, groups=dw_channels)
        pw = _seq_conv_bn_relu(dw_channels, out_channels, 1, 1, 0)
        self.conv = nn.Sequential(*dw, *pw)


class _DWConv(_Container):
    """models/fast_scnn.py:82-92."""

    def __init__(self, dw_channels, out_channels, stride=1, **kwargs):
        super().__init__()
        self.conv = _seq_conv_bn_relu(dw_channels, out_channels, 3, stride, 1, groups=dw_channels)


class LinearBottleneck(_Container):
    """models/fast_scnn.py:95-115 (t = 6, shortcut iff stride 1 and Cin == Cout)."""

    def __init__(self, in_channels, out_channels, t=6, stride=2, **kwargs):
        super().__init__()
        self.use_shortcut = stride == 1 and in_channels == out_channels
        e = in_channels * t
        self.block = nn.Sequential(_ConvBNReLU(in_channels, e, 1), _DWConv(e, e, stride),
                                   nn.Conv2d(e, out_channels, 1, bias=False),
                                   nn.BatchNorm2d(out_channels))


class PyramidPooling(_Container):
    """models/fast_scnn.py:118-145."""

    def __init__(self, in_channels, out_channels, **kwargs):
        super().__init__()
        inter = int(in_channels / 4)
        for i in range(1, 5):
            setattr(self, "conv%d" % i, _ConvBNReLU(in_channels, inter, 1))
        self.out = _ConvBNReLU(in_channels * 2, out_channels, 1)


class LearningToDownsample(_Container):
    """models/fast_scnn.py:148-161."""

    def __init__(self, dw_channels1=32, dw_channels2=48, out_channels=64, **kwargs):
        super().__init__()
        self.conv = _ConvBNReLU(3, dw_channels1, 3, 2)
        self.dsconv1 = _DSConv(dw_channels1, dw_channels2, 2)
        self.dsconv2 = _DSConv(dw_channels2, out_channels, 2)


class GlobalFeatureExtractor(_Container):
    """models/fast_scnn.py:164-187."""

    def __init__(self, in_channels=64, block_channels=(64, 96, 128), out_channels=128, t=6,
                 num_blocks=(3, 3, 3), **kwargs):
        super().__init__()
        strides = (2, 2, 1)
        cin = in_channels
        for i, (cout, n, s) in enumerate(zip(block_channels, num_blocks, strides)):
            blocks = [LinearBottleneck(cin if j == 0 else cout, cout, t, s if j == 0 else 1)
                      for j in range(n)]
            setattr(self, "bottleneck%d" % (i + 1), nn.Sequential(*blocks))
            cin = cout
        self.ppm = PyramidPooling(block_channels[2], out_channels)


class FeatureFusionModule(_Container):
    """models/fast_scnn.py:190-218."""

    def __init__(self, highter_in_channels, lower_in_channels, out_channels, scale_factor=4,
                 **kwargs):
        super().__init__()
        self.scale_factor = scale_factor
        self.dwconv = _DWConv(lower_in_channels, out_channels, 1)
        self.conv_lower_res = nn.Sequential(nn.Conv2d(out_channels, out_channels, 1),
                                            nn.BatchNorm2d(out_channels))
        self.conv_higher_res = nn.Sequential(nn.Conv2d(highter_in_channels, out_channels, 1),
                                             nn.BatchNorm2d(out_channels))
        self.relu = nn.ReLU(True)


class Classifer(_Container):
    """models/fast_scnn.py:221-237 (reference spelling kept)."""

    def __init__(self, dw_channels, num_classes, stride=1, **kwargs):
        super().__init__()
        self.dsconv1 = _DSConv(dw_channels, dw_channels, stride)
        self.dsconv2 = _DSConv(dw_channels, dw_channels, stride)
        self.conv = nn.Sequential(nn.Dropout(0.1), nn.Conv2d(dw_channels, num_classes, 1))


# ---------------------------------------------------------------------------------------------
# native network handle + plans
# ---------------------------------------------------------------------------------------------
class _Native:
    """Owns the C++ fscnn_net and a cache of fscnn_plan handles."""

    def __init__(self, num_classes, aux):
        lib = _lib.load()
        h = _lib.c_vp()
        _lib.check(lib.fscnn_net_create(num_classes, int(aux), _lib.ctypes.byref(h)),
                   "fscnn_net_create")
        self.h = h
        self.lib = lib
        n, tot = _lib.c_int(), _lib.c_ll()
        _lib.check(lib.fscnn_net_param_count(h, _lib.ctypes.byref(n), _lib.ctypes.byref(tot)))
        self.p_total = tot.value
        self.params = [self._info("fscnn_net_param_info", i) for i in range(n.value)]
        nb, rtot, nbn = _lib.c_int(), _lib.c_ll(), _lib.c_int()
        _lib.check(lib.fscnn_net_buffer_count(h, _lib.ctypes.byref(nb), _lib.ctypes.byref(rtot),
                                              _lib.ctypes.byref(nbn)))
        self.r_total, self.n_bn = rtot.value, nbn.value
        self.buffers = [self._info("fscnn_net_buffer_info", i) for i in range(nb.value)]
        self.stage_ranges = []
        for s in range(4):
            b, e = _lib.c_ll(), _lib.c_ll()
            _lib.check(lib.fscnn_net_stage_range(h, s, _lib.ctypes.byref(b), _lib.ctypes.byref(e)))
            self.stage_ranges.append((b.value, e.value))
        self.plans = {}
        self._lock = threading.Lock()

    def _info(self, fn, i):
        name, off, numel = _lib.c_char_p(), _lib.c_ll(), _lib.c_ll()
        _lib.check(getattr(self.lib, fn)(self.h, i, _lib.ctypes.byref(name), _lib.ctypes.byref(off),
                                         _lib.ctypes.byref(numel)), fn)
        return name.value.decode(), off.value, numel.value

    def plan(self, N, H, W, dtype_code, train, device=None):
        """Plan of one (N, H, W, dtype, mode) on one device.  Plans are per device (each owns its
        side stream and graph cache) and created under a lock: DataParallel's worker threads
        (train.py:170-171 -> parallel_apply) reach here concurrently."""
        key = (None if device is None else device.index, N, H, W, dtype_code, int(train))
        p = self.plans.get(key)
        if p is not None:
            return p
        with self._lock:
            p = self.plans.get(key)
            if p is not None:
                return p
            h = _lib.c_vp()
            _lib.check(self.lib.fscnn_plan_create(self.h, N, H, W, dtype_code, int(train),
                                                  _lib.ctypes.byref(h)), "fscnn_plan_create")
            fw, bw = _lib.c_ll(), _lib.c_ll()
            _lib.check(self.lib.fscnn_plan_workspace(h, _lib.ctypes.byref(fw),
                                                     _lib.ctypes.byref(bw)))
            p = (h, fw.value, bw.value)
            self.plans[key] = p
        return p

    def __del__(self):
        try:
            for h, _, _ in self.plans.values():
                self.lib.fscnn_plan_destroy(h)
            self.lib.fscnn_net_destroy(self.h)
        except Exception:
            pass


class _Shared:
    """State a FastSCNN shares with its DataParallel replicas: ``replicate()``
    (torch/nn/parallel/replicate.py, driven by train.py:170-171) shallow-copies the module's
    ``__dict__``, so every replica sees this same object — one native net handle and one plan
    cache for the whole wrapper.  A deep copy / pickle of the model starts a fresh one."""

    def __init__(self):
        self.native = None
        self.lock = threading.Lock()

    def __deepcopy__(self, memo):
        return _Shared()

    def __getstate__(self):
        return {}

    def __setstate__(self, state):
        self.__init__()


MODE_EVAL, MODE_TRAIN, MODE_EVAL_GRAD = 0, 1, 2  # plan modes (include/fastscnn.h fscnn_plan_create)


class _FastSCNNFunction(torch.autograd.Function):
    """Whole-network forward / staged backward; grads are views of one flat arena.

    train mode: the training forward keeps its workspace (every pre-BN tensor) for the backward.
    eval mode (the reference module stays differentiable: models/fast_scnn.py:33-46 has no
    no_grad, and eval.py:43 calls it with grad enabled): the forward is the fused inference path
    (same speed and memory as under no_grad), and the backward first recomputes the forward as a
    differentiable-inference plan (mode 2: every BatchNorm normalised by its running statistics,
    Dropout off) and then runs the staged backward of that plan.  The parameters are saved for
    the backward, so autograd refuses one that changed in place in between, as it would for the
    reference's convolution weights."""

    @staticmethod
    def forward(ctx, x, model, ar, *params):
        ctx.model, ctx.ar = model, ar
        if model.training:
            outs, ws, seed, dt, xc = model._run_forward(x, MODE_TRAIN, ar=ar)
            ctx.mode, ctx.ws, ctx.seed, ctx.dt = MODE_TRAIN, ws, seed, dt
        else:
            outs, _, _, dt, xc = model._run_forward(x, MODE_EVAL, ar=ar)
            ctx.mode, ctx.ws, ctx.seed, ctx.dt = MODE_EVAL_GRAD, None, 0, dt
            # the backward recomputes this forward from the running statistics: remember their
            # version (a train-mode forward or a load_state_dict in between bumps it)
            ctx.r_version = ar["R"]._version
        ctx.x_dtype = x.dtype
        # the converted dense NCHW fp32/bf16 copy the forward read, not the caller's tensor: the
        # conv0 weight gradient re-reads it as dense NCHW (channels_last / fp16 / expanded inputs)
        ctx.save_for_backward(xc, *params)
        return outs if len(outs) > 1 else outs[0]

    @staticmethod
    def backward(ctx, *gouts):
        x = ctx.saved_tensors[0]  # (autograd checks the saved parameters' versions here)
        gaux = gouts[1] if len(gouts) > 1 else None
        model, ws = ctx.model, ctx.ws
        if ctx.mode == MODE_EVAL_GRAD:
            if ctx.ar["R"]._version != ctx.r_version:
                raise RuntimeError(
                    "one of the variables needed for gradient computation has been modified by an "
                    "inplace operation: the BatchNorm running statistics changed (a train-mode "
                    "forward or a state_dict load) between this eval-mode forward and its backward")
            # (in the forward's arithmetic: autocast is not active where autograd runs backward)
            _, ws, _, _, _ = model._run_forward(x, MODE_EVAL_GRAD, ar=ctx.ar, dt=ctx.dt)
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        grads = model._run_backward(gouts[0], x, ws, ctx.seed, ctx.dt, ctx.ar, gaux=gaux,
                                    mode=ctx.mode, dx=dx)
        ctx.ws = ctx.ar = None
        if dx is not None and dx.dtype != ctx.x_dtype:
            dx = dx.to(ctx.x_dtype)
        return (dx, None, None) + tuple(grads)


class _FastSCNNLossFunction(torch.autograd.Function):
    """Fused train step head: loss = CE(upsample(logits_lowres), target) at low resolution."""

    @staticmethod
    def forward(ctx, x, target, ignore_index, model, ar, *params):
        loss2, ws, seed, dt, xc = model._run_forward_loss(x, target, ignore_index, ar)
        ctx.model, ctx.ar = model, ar
        ctx.ws, ctx.seed, ctx.dt, ctx.loss2 = ws, seed, dt, loss2
        ctx.x_dtype = x.dtype
        ctx.save_for_backward(xc, *params)
        # the mean of the (mean, count) pair the head wrote, as a tensor sharing its storage but
        # not an autograd view (a view created here would refuse the in-place ops the reference's
        # loss tensor allows: loss /= accum_steps); the backward reads only the count, loss2[1]
        out = torch.empty((), dtype=loss2.dtype, device=loss2.device)
        return out.set_(loss2.untyped_storage(), loss2.storage_offset(), (), ())

    @staticmethod
    def backward(ctx, gloss):
        x = ctx.saved_tensors[0]
        g = gloss.to(torch.float32).reshape(1).contiguous()
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        grads = ctx.model._run_backward(None, x, ctx.ws, ctx.seed, ctx.dt, ctx.ar, gloss=g,
                                        loss2=ctx.loss2, dx=dx)
        ctx.ws = ctx.ar = None
        if dx is not None and dx.dtype != ctx.x_dtype:
            dx = dx.to(ctx.x_dtype)
        return (dx, None, None, None, None) + tuple(grads)


class FastSCNN(nn.Module):
    """Fast-SCNN (models/fast_scnn.py:16-46) on the MI355X HIP path."""

    def __init__(self, num_classes, aux=False, **kwargs):
        super().__init__()
        self.aux = aux
        self.learning_to_downsample = LearningToDownsample(32, 48, 64)
        self.global_feature_extractor = GlobalFeatureExtractor(64, [64, 96, 128], 128, 6, [3, 3, 3])
        self.feature_fusion = FeatureFusionModule(64, 128, 128)
        self.classifier = Classifer(128, num_classes)
        if self.aux:
            self.auxlayer = nn.Sequential(nn.Conv2d(64, 32, 3, padding=1, bias=False),
                                          nn.BatchNorm2d(32), nn.ReLU(True), nn.Dropout(0.1),
                                          nn.Conv2d(32, num_classes, 1))
        self.num_classes = num_classes
        object.__setattr__(self, "_shared", _Shared())
        object.__setattr__(self, "_arena", None)
        object.__setattr__(self, "grad_stage_hook", None)

    # ---- arenas ----------------------------------------------------------------------------
    def native(self):
        sh = self._shared
        if sh.native is None:
            with sh.lock:
                if sh.native is None:
                    nat = _Native(self.num_classes, self.aux)
                    names = [n for n, _ in self._named_params()]
                    if names != [p[0] for p in nat.params]:
                        raise RuntimeError("FastSCNN: parameter table mismatch with the native "
                                           "executor")
                    sh.native = nat
        return sh.native

    def _is_dp_replica(self):
        return bool(getattr(self, "_is_replica", False))

    def _named_params(self):
        """named_parameters() of the module, or of a DataParallel replica: ``replicate()`` keeps
        a replica's (non-leaf, broadcast) parameter tensors as plain attributes and lists them in
        each submodule's ``_former_parameters`` in ``_parameters`` order."""
        if not self._is_dp_replica():
            return list(self.named_parameters())
        out = []
        for mname, m in self.named_modules():
            for k, t in getattr(m, "_former_parameters", {}).items():
                if t is not None:
                    out.append((mname + "." + k if mname else k, t))
        return out

    def _apply(self, fn, recurse=True):
        r = super()._apply(fn, recurse)
        object.__setattr__(self, "_arena", None)
        return r

    def _pack_arena(self):
        """Re-home params / buffers into the executor's flat arenas on their current device."""
        nat = self.native()
        params = list(self.parameters())
        dev = params[0].device
        P = torch.zeros(nat.p_total, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for p, (_, off, numel) in zip(params, nat.params):
                if p.numel() != numel or p.dtype != torch.float32:
                    raise RuntimeError("FastSCNN: parameter %s has unexpected shape/dtype" % (_,))
                P[off:off + numel].copy_(p.detach().reshape(-1))
                p.data = P[off:off + numel].view(p.shape)
            R = torch.zeros(nat.r_total, dtype=torch.float32, device=dev)
            NBT = torch.zeros(nat.n_bn, dtype=torch.int64, device=dev)
            mods = dict(self.named_modules())
            for name, off, numel in nat.buffers:
                mname, bname = name.rsplit(".", 1)
                m = mods[mname]
                cur = m._buffers[bname]
                if bname == "num_batches_tracked":
                    NBT[off].copy_(cur.reshape(()))
                    m._buffers[bname] = NBT[off]
                else:
                    R[off:off + numel].copy_(cur.reshape(-1))
                    m._buffers[bname] = R[off:off + numel]
        arena = {"P": P, "R": R, "NBT": NBT, "params": params,
                 "ptrs": (params[0].data_ptr(), params[-1].data_ptr())}
        object.__setattr__(self, "_arena", arena)
        return arena

    def arena(self):
        a = self._arena
        params = None
        if a is not None:
            params = a["params"]
            if (params[0].data_ptr(), params[-1].data_ptr()) != a["ptrs"] or \
                    params[0].data_ptr() != a["P"].data_ptr():
                a = None
        if a is None:
            a = self._pack_arena()
        return a

    def _replica_arena(self, dev):
        """Arenas of a DataParallel replica (train.py:170-171) on ``dev``.

        Replica 0 aliases the module's own tensors (``comm.broadcast_coalesced`` returns the
        source device's inputs), so its parameters and buffers already are views of the packed
        arenas.  Any other replica holds broadcast copies: they are packed into fresh arenas on
        its device for this call (one multi-tensor copy each), and the running statistics the
        train forward updates are written back into the replica's own buffers, as aten's
        batch_norm would have updated them.  ``params`` are always the replica's tensors, so the
        autograd Function's gradients flow back through ``Broadcast`` (reduce-add to cuda:0)."""
        nat = self.native()
        params = [t for _, t in self._named_params()]
        if len(params) != len(nat.params):
            raise RuntimeError("FastSCNN replica: %d parameters, executor expects %d"
                               % (len(params), len(nat.params)))
        mods = dict(self.named_modules())
        bufs = []
        for name, off, numel in nat.buffers:
            mname, bname = name.rsplit(".", 1)
            bufs.append((mods[mname]._buffers[bname], off, numel, bname == "num_batches_tracked"))
        m = self._arena  # the module's arenas, as they were when replicate() copied __dict__
        if m is not None and m["P"].device == dev:
            P, R, NBT = m["P"], m["R"], m["NBT"]
            pb, rb, nb = P.data_ptr(), R.data_ptr(), NBT.data_ptr()
            alias = all(t.data_ptr() == pb + 4 * off
                        for t, (_, off, _n) in zip((params[0], params[-1]),
                                                   (nat.params[0], nat.params[-1])))
            alias = alias and all(t.data_ptr() == (nb + 8 * off if isn else rb + 4 * off)
                                  for t, off, _n, isn in (bufs[0], bufs[-1], bufs[1]))
            if alias:
                return {"P": P, "R": R, "NBT": NBT, "params": params, "writeback": None}
        with torch.no_grad():
            P = torch.zeros(nat.p_total, dtype=torch.float32, device=dev)
            R = torch.zeros(nat.r_total, dtype=torch.float32, device=dev)
            NBT = torch.zeros(nat.n_bn, dtype=torch.int64, device=dev)
            pv = [P[off:off + numel] for _, off, numel in nat.params]
            torch._foreach_copy_(pv, [p.detach().reshape(-1) for p in params])
            rv = [NBT[off] if isn else R[off:off + numel] for _, off, numel, isn in bufs]
            bt = [b if isn else b.reshape(-1) for b, _o, _n, isn in bufs]
            torch._foreach_copy_(rv, bt)
        return {"P": P, "R": R, "NBT": NBT, "params": params, "writeback": (bt, rv)}

    def _exec_arena(self, dev):
        return self._replica_arena(dev) if self._is_dp_replica() else self.arena()

    @staticmethod
    def _writeback(ar):
        """Running statistics of a replica's packed copy -> the replica's own buffers."""
        wb = ar.get("writeback")
        if wb is not None:
            with torch.no_grad():
                torch._foreach_copy_(wb[0], wb[1])

    def load_state_dict(self, state_dict, strict=True, assign=False):
        r = super().load_state_dict(state_dict, strict=strict, assign=assign)
        if assign:
            object.__setattr__(self, "_arena", None)
        return r

    # ---- execution ----------------------------------------------------------------------------
    def _compute_dtype(self, x, train):
        """Arithmetic of the call, as the reference's convolutions would run it.

        * Under ``torch.autocast("cuda")`` (train.py:269's ``torch.cuda.amp.autocast()``, fp16 by
          default; test_specific_images.py:121's inference): autocast's dtype — fp16 unless the
          caller asked for bf16.  16-bit activations and logits, fp32 master weights, BN
          statistics, accumulation and weight gradients.
        * Otherwise the input's dtype: fp32 (cfg1 / cfg2), bf16 (cfg3's arithmetic), fp16
          (cfg5's fp16 images).
        ``train`` does not change the choice: every dtype has forward and backward kernels."""
        if torch.is_autocast_enabled("cuda"):
            dt = torch.get_autocast_dtype("cuda")
            if dt in (torch.float16, torch.bfloat16):
                return dt
            raise RuntimeError("FastSCNN: unsupported autocast dtype %s" % (dt,))
        if x.dtype in (torch.float32, torch.bfloat16, torch.float16):
            return x.dtype
        raise RuntimeError("FastSCNN: unsupported input dtype %s" % (x.dtype,))

    @staticmethod
    def _input(x):
        """Dense NCHW copy of the input in a dtype conv0 reads (fp32 / bf16 / fp16)."""
        if x.dtype not in (torch.float32, torch.bfloat16, torch.float16):
            x = x.float()
        return x.contiguous()

    def _momentum(self):
        m = self.learning_to_downsample.conv.conv[1].momentum
        if m is None:
            raise RuntimeError("FastSCNN: BatchNorm momentum=None (cumulative) is not supported")
        return float(m)

    def _dropout_p(self):
        return float(self.classifier.conv[0].p)

    def _run_forward(self, x, mode, ar=None, dt=None):
        """One native forward; mode: MODE_EVAL (0), MODE_TRAIN (1), MODE_EVAL_GRAD (2); dt: the
        arithmetic (default: _compute_dtype)."""
        train = mode == MODE_TRAIN
        if x.dim() != 4 or x.shape[1] != 3:
            raise RuntimeError("FastSCNN: expected input [N, 3, H, W], got %s" % (tuple(x.shape),))
        if not x.is_cuda:
            raise RuntimeError("FastSCNN: the HIP path needs a ROCm device tensor (got %s); "
                               "move the model and input to 'cuda'" % (x.device,))
        nat = self.native()
        if ar is None:
            ar = self._exec_arena(x.device)
        if ar["P"].device != x.device:
            raise RuntimeError("FastSCNN: input on %s but parameters on %s"
                               % (x.device, ar["P"].device))
        N, _, H, W = x.shape
        if H < 32 or W < 32:
            raise RuntimeError("FastSCNN: input %dx%d too small (needs >= 32x32)" % (H, W))
        if dt is None:
            dt = self._compute_dtype(x, train)
        x = self._input(x)
        if train and N < 2:
            # the reference raises from the PPM 1x1 BatchNorm in train mode (SURVEY §0 trap 5)
            raise ValueError("Expected more than 1 value per channel when training, got input "
                             "size torch.Size([1, 32, 1, 1])")
        plan, fw, _ = nat.plan(N, H, W, _lib.dtype_code(dt), mode, x.device)
        ws = torch.empty(max(fw, 1), dtype=torch.uint8, device=x.device)
        out_dt = dt  # (autocast: the reference's final F.interpolate returns fp16 logits)
        out = torch.empty((N, self.num_classes, H, W), dtype=out_dt, device=x.device)
        aux_out = torch.empty_like(out) if self.aux else None
        p = self._dropout_p() if train else 0.0
        seed = 0
        if train and p > 0:
            fixed = getattr(self, "_dropout_seed", None)  # tests pin the mask (oracle parity)
            seed = int(fixed) if fixed is not None else int(torch.randint(0, 2 ** 62, (1,)).item())
        rest = (_lib.dtype_code(dt), _lib.ptr(ar["P"]), _lib.ptr(ar["R"]), _lib.ptr(ar["NBT"]),
                _lib.ptr(ws), _lib.c_ull(seed), _lib.c_float(p), _lib.c_float(self._momentum()),
                _lib.stream_ptr(x.device))
        with torch.cuda.device(x.device):
            if self.aux:  # models/fast_scnn.py:42-45
                _lib.call("fscnn_forward_aux", plan, _lib.ptr(x), _lib.dtype_code(x.dtype),
                          _lib.ptr(out), _lib.ptr(aux_out), _lib.dtype_code(out_dt), *rest[1:])
            else:
                _lib.call("fscnn_forward", plan, _lib.ptr(x), _lib.dtype_code(x.dtype),
                          _lib.ptr(out), _lib.dtype_code(out_dt), *rest[1:])
        if train:
            self._writeback(ar)
            # the running statistics changed: an eval-mode graph recorded before this forward
            # must not backpropagate through them (_FastSCNNFunction.backward checks)
            torch.autograd.graph.increment_version(ar["R"])
        if getattr(self, "_keep_ws", False):
            self._debug = {"plan": plan, "ws": ws, "dt": dt}
        return ((out, aux_out) if self.aux else (out,)), ws, seed, dt, x

    def predict(self, x, dtype=torch.int64):
        """``torch.argmax(self(x)[0], 1)`` of an eval-mode model (eval.py:43-45, demo.py:43-48)
        without the upsampled logits: the final bilinear upsample and the argmax over classes run
        as one kernel that writes only the labels (int64 like torch.argmax, or uint8)."""
        if self.training:
            raise RuntimeError("predict is the inference path; call model.eval() first")
        if dtype not in (torch.int64, torch.uint8):
            raise RuntimeError("predict: labels are int64 or uint8, not %s" % (dtype,))
        if x.dim() != 4 or x.shape[1] != 3:
            raise RuntimeError("FastSCNN: expected input [N, 3, H, W], got %s" % (tuple(x.shape),))
        if not x.is_cuda:
            raise RuntimeError("FastSCNN.predict: the HIP path needs a ROCm device tensor")
        nat = self.native()
        ar = self._exec_arena(x.device)
        N, _, H, W = x.shape
        if H < 32 or W < 32:
            raise RuntimeError("FastSCNN: input %dx%d too small (needs >= 32x32)" % (H, W))
        dt = self._compute_dtype(x, False)
        x = self._input(x)
        plan, fw, _ = nat.plan(N, H, W, _lib.dtype_code(dt), False, x.device)
        ws = torch.empty(max(fw, 1), dtype=torch.uint8, device=x.device)
        labels = torch.empty((N, H, W), dtype=dtype, device=x.device)
        with torch.cuda.device(x.device):
            _lib.call("fscnn_predict", plan, _lib.ptr(x), _lib.dtype_code(x.dtype),
                      _lib.ptr(labels), 1 if dtype == torch.uint8 else 0, _lib.ptr(ar["P"]),
                      _lib.ptr(ar["R"]), _lib.ptr(ar["NBT"]), _lib.ptr(ws),
                      _lib.stream_ptr(x.device))
        if getattr(self, "_keep_ws", False):
            self._debug = {"plan": plan, "ws": ws, "dt": dt}
        return labels

    def debug_buffer(self, name):
        """Tensor view of a named plan buffer of the last forward/backward (set ``_keep_ws``).

        Debug / stage-level parity helper: returns [rows, cols] in the compute dtype."""
        d = self._debug
        off, rows, cols, ld, inb = (_lib.c_ll(), _lib.c_ll(), _lib.c_int(), _lib.c_int(),
                                    _lib.c_int())
        _lib.check(_lib.load().fscnn_plan_buffer(d["plan"], name.encode(), _lib.ctypes.byref(off),
                                                 _lib.ctypes.byref(rows), _lib.ctypes.byref(cols),
                                                 _lib.ctypes.byref(ld), _lib.ctypes.byref(inb)),
                   "fscnn_plan_buffer")
        base = d["bws"] if inb.value else d["ws"]
        dt = d["dt"] if not name.endswith((".scale", ".shift", ".mean", ".invstd")) else torch.float32
        esz = torch.tensor([], dtype=dt).element_size()
        n = (rows.value - 1) * ld.value + cols.value
        flat = base[off.value:off.value + n * esz].view(dt)
        return flat.as_strided((rows.value, cols.value), (ld.value, 1))

    def _run_forward_loss(self, x, target, ignore_index, ar):
        if self.aux:
            raise RuntimeError("forward_loss: the fused loss head covers the main output only; "
                               "with aux=True use MixSoftmaxCrossEntropyLoss(aux=True)"
                               "(model(x), target)")
        if not x.is_cuda or not target.is_cuda:
            raise RuntimeError("FastSCNN.forward_loss: the HIP path needs ROCm device tensors")
        nat = self.native()
        N, _, H, W = x.shape
        if tuple(target.shape) != (N, H, W):
            raise RuntimeError("forward_loss: target %s does not match input %s"
                               % (tuple(target.shape), tuple(x.shape)))
        if N < 2:
            raise ValueError("Expected more than 1 value per channel when training, got input "
                             "size torch.Size([1, 32, 1, 1])")
        dt = self._compute_dtype(x, True)
        x = self._input(x)
        target = target.to(torch.int64).contiguous()
        from . import loss as _loss
        if _loss.CHECK_TARGETS:
            _loss.check_targets(target, self.num_classes, ignore_index)
        plan, fw, _ = nat.plan(N, H, W, _lib.dtype_code(dt), True, x.device)
        ws = torch.empty(max(fw, 1), dtype=torch.uint8, device=x.device)
        loss2 = torch.empty(2, dtype=torch.float32, device=x.device)
        p = self._dropout_p()
        seed = 0
        if p > 0:
            fixed = getattr(self, "_dropout_seed", None)
            seed = int(fixed) if fixed is not None else int(torch.randint(0, 2 ** 62, (1,)).item())
        with torch.cuda.device(x.device):
            _lib.call("fscnn_forward_loss", plan, _lib.ptr(x), _lib.dtype_code(x.dtype),
                      _lib.ptr(target), int(ignore_index), _lib.ptr(loss2), _lib.ptr(ar["P"]),
                      _lib.ptr(ar["R"]), _lib.ptr(ar["NBT"]), _lib.ptr(ws), _lib.c_ull(seed),
                      _lib.c_float(p), _lib.c_float(self._momentum()), _lib.stream_ptr(x.device))
        self._writeback(ar)
        torch.autograd.graph.increment_version(ar["R"])
        if getattr(self, "_keep_ws", False):
            self._debug = {"plan": plan, "ws": ws, "dt": dt}
        return loss2, ws, seed, dt, x

    def forward_loss(self, x, target, ignore_index=-1):
        """Fused train-step head: ``criterion(self(x)[0], target)`` of train.py:270-271 for
        ``nn.CrossEntropyLoss(ignore_index)`` (utils/loss.py:103-124), computed at the low-res
        logit resolution without materialising full-resolution logits.  Same loss and gradients
        as the unfused path (tests/test_gpu_model.py); requires train mode."""
        if not self.training:
            raise RuntimeError("forward_loss is the training step; call model.train() first")
        if not x.is_cuda:
            raise RuntimeError("FastSCNN.forward_loss: the HIP path needs ROCm device tensors")
        ar = self._exec_arena(x.device)
        return _FastSCNNLossFunction.apply(x, target, ignore_index, self, ar, *ar["params"])

    def _run_backward(self, gout, x, ws, seed, dt, ar, gloss=None, loss2=None, gaux=None,
                      mode=MODE_TRAIN, dx=None):
        """The staged native backward of a MODE_TRAIN / MODE_EVAL_GRAD forward whose workspace
        is ``ws``; parameter gradients are views of one flat arena G, and ``dx`` (dense NCHW,
        the dtype of ``x``) receives the input gradient when given."""
        nat = self.native()
        N, _, H, W = x.shape
        plan, _, bw = nat.plan(N, H, W, _lib.dtype_code(dt), mode, x.device)
        if gout is not None:
            gout = gout.to(dt).contiguous()
        if self.aux and gloss is None:
            gaux = torch.zeros_like(gout) if gaux is None else gaux.to(dt).contiguous()
        # every element of every parameter's gradient is written by the backward (a reduction,
        # a BN finish or the PPM kernel; tests/test_gpu_model.py fills G with NaN to check), so
        # the arena is not zeroed; only the 64-B alignment gaps between tensors are left as is
        G = torch.empty(nat.p_total, dtype=torch.float32, device=x.device)
        if getattr(self, "_debug_fill_grads", None) is not None:
            G.fill_(self._debug_fill_grads)
        bws = torch.empty(max(bw, 1), dtype=torch.uint8, device=x.device)
        p = self._dropout_p() if mode == MODE_TRAIN else 0.0
        if getattr(self, "_keep_ws", False):
            self._debug["bws"] = bws
        hook = self.grad_stage_hook
        if hook is None:
            # one native call for the four stages: their weight-gradient reductions run once at
            # its end, so the main stream does not wait for the side stream between stages
            with torch.cuda.device(x.device):
                self._backward_stage(plan, (0, 3), gout, gaux, gloss, loss2, x, ar, G, ws, bws,
                                     seed, p, dx)
        else:
            for s in range(4):
                with torch.cuda.device(x.device):
                    self._backward_stage(plan, (s, s), gout, gaux, gloss, loss2, x, ar, G, ws,
                                         bws, seed, p, dx)
                b, e = nat.stage_ranges[s]
                hook(s, G, b, e)
        return [G[off:off + numel].view(prm.shape)
                for prm, (_, off, numel) in zip(ar["params"], nat.params)]

    def _backward_stage(self, plan, stages, gout, gaux, gloss, loss2, x, ar, G, ws, bws, seed, p,
                        dx=None):
        s0, s1 = stages  # backward stages s0 .. s1 (0: head ... 3: LearningToDownsample)
        if dx is not None:  # the general entry point: also writes the input gradient (stage 3)
            _lib.call("fscnn_backward_dx", plan, _lib.ptr(gout), _lib.ptr(gaux), _lib.ptr(gloss),
                      _lib.ptr(loss2), _lib.ptr(x), _lib.dtype_code(x.dtype), _lib.ptr(dx),
                      _lib.dtype_code(dx.dtype), _lib.ptr(ar["P"]), _lib.ptr(G), _lib.ptr(ws),
                      _lib.ptr(bws), _lib.c_ull(seed), _lib.c_float(p), s0, s1,
                      _lib.stream_ptr(x.device))
        elif gloss is None and self.aux:
            _lib.call("fscnn_backward_aux", plan, _lib.ptr(gout), _lib.ptr(gaux), _lib.ptr(x),
                      _lib.dtype_code(x.dtype), _lib.ptr(ar["P"]), _lib.ptr(G), _lib.ptr(ws),
                      _lib.ptr(bws), _lib.c_ull(seed), _lib.c_float(p), s0, s1,
                      _lib.stream_ptr(x.device))
        elif gloss is None:
            _lib.call("fscnn_backward", plan, _lib.ptr(gout), _lib.ptr(x),
                      _lib.dtype_code(x.dtype), _lib.ptr(ar["P"]), _lib.ptr(G), _lib.ptr(ws),
                      _lib.ptr(bws), _lib.c_ull(seed), _lib.c_float(p), s0, s1,
                      _lib.stream_ptr(x.device))
        else:
            _lib.call("fscnn_backward_loss", plan, _lib.ptr(gloss), _lib.ptr(loss2), _lib.ptr(x),
                      _lib.dtype_code(x.dtype), _lib.ptr(ar["P"]), _lib.ptr(G), _lib.ptr(ws),
                      _lib.ptr(bws), _lib.c_ull(seed), _lib.c_float(p), s0, s1,
                      _lib.stream_ptr(x.device))

    def _needs_graph(self, x):
        """Whether this call is differentiable, as the reference's would be: train mode with
        grad enabled (the training step), or any mode when autograd would record the call (an
        input or a parameter requires grad).  eval() under torch.no_grad() is the inference path."""
        if not torch.is_grad_enabled():
            return False
        if self.training or x.requires_grad:
            return True
        return any(p.requires_grad for p in self.parameters())

    def forward(self, x):
        mode = MODE_TRAIN if self.training else MODE_EVAL
        if self._needs_graph(x):
            if not x.is_cuda:
                self._run_forward(x, mode)  # raises the device error
            ar = self._exec_arena(x.device)
            out = _FastSCNNFunction.apply(x, self, ar, *ar["params"])
            return tuple(out) if self.aux else (out,)
        return self._run_forward(x, mode)[0]


def get_fast_scnn(dataset="citys", pretrained=False, root="./weights", map_cpu=False, **kwargs):
    """models/fast_scnn.py:240-256 without the torchvision-importing data_loader lookup."""
    acronyms = {"pascal_voc": "voc", "pascal_aug": "voc", "ade20k": "ade", "coco": "coco",
                "citys": "citys", "tusimple": "tusimple"}
    if dataset not in NUM_CLASS:
        raise KeyError(dataset)
    model = FastSCNN(NUM_CLASS[dataset], **kwargs)
    if pretrained:
        path = os.path.join(root, "fast_scnn_%s.pth" % acronyms[dataset])
        sd = torch.load(path, map_location="cpu" if map_cpu else None, weights_only=True)
        model.load_state_dict(strip_module_prefix(sd))
    return model


def strip_module_prefix(state_dict):
    """Checkpoints saved from the DataParallel / DistributedFastSCNN wrapper (train.py:449 saves
    ``model.state_dict()`` with a ``module.`` prefix) load into a bare FastSCNN (SURVEY §8(f) row
    4); other keys are left as they are."""
    if all(k.startswith("module.") for k in state_dict):
        return type(state_dict)((k[len("module."):], v) for k, v in state_dict.items())
    return state_dict
