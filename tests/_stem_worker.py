"""Worker for tests/test_gpu_switches.py::test_stem_fused_bit_identical (fresh process: the
executor reads FSCNN_STEM_FUSED once).  Eval forwards (no_grad) over the image dtypes and map
sizes the fused inference stem (csrc/stem.hip) handles -- partial edge tiles included -- saving
every output, plus the number of stem launches the library's profiler saw in the first case.
With ``--dsconv``: the same for the fused classifier DSConvs (csrc/dsconv.hip,
FSCNN_DSCONV_FUSED) over maps whose classifier M = N x H/8 x W/8 >= 4096.  With ``--ppm``: the
inference PPM branch convs in one launch (csrc/ppm.hip, FSCNN_PPM_FUSED) over batches whose bins
leave partial 16-row tiles.

    python tests/_stem_worker.py OUT.npz [--dsconv | --ppm]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# (fp32: the unfused dsconv1.pw takes the streaming GEMM -- whose six-product order the stem
# reproduces -- at M >= 4096 dsconv1 pixels only; below that the tiled GEMM sums the split
# products in another order, equal to fp32 rounding but not bit for bit)
CASES = [  # (name, classes, shape, image dtype, autocast dtype)
    ("fp32", 19, (2, 3, 256, 256), "float32", None),
    ("fp32_odd", 19, (1, 3, 262, 332), "float32", None),  # 65 x 83 outputs: partial tiles
    ("bf16", 19, (2, 3, 96, 160), "bfloat16", None),
    ("fp16_c2", 2, (2, 3, 120, 160), "float16", None),
    ("autocast16", 19, (1, 3, 64, 96), "float32", "float16"),
    ("fp32_unaligned", 19, (1, 3, 66, 98), "float32", None),  # W % 4 != 0: unfused either way
]
PK_STEM = 17
# (the classifier runs at H/8 x W/8: M >= 4096 for the unfused pointwise to take the streaming
# GEMM whose MFMA order the fused DSConv reproduces)
DS_CASES = [
    ("fp32", 19, (2, 3, 512, 512), "float32", None),
    ("fp32_odd", 19, (1, 3, 520, 1048), "float32", None),  # 65 x 131: partial strips and segments
    ("bf16", 19, (1, 3, 512, 1024), "bfloat16", None),
    ("fp16_c2", 2, (1, 3, 480, 640), "float16", None),
    ("autocast16", 19, (1, 3, 520, 1048), "float32", "float16"),
]
PK_DSCONV = 18
# (the PPM branches have M = k*k*N rows < 4096, where the unfused pointwise takes the tiled GEMM
# whose k order the fused launch reproduces)
PPM_CASES = [
    ("fp32", 19, (2, 3, 256, 512), "float32", None),
    ("fp32_n3", 19, (3, 3, 320, 416), "float32", None),  # 3 / 12 / 27 / 108 rows
    ("fp32_n8", 19, (8, 3, 256, 256), "float32", None),  # 8 / 32 / 72 / 288 rows (cfg2's bins)
    ("bf16", 19, (3, 3, 192, 256), "bfloat16", None),
    ("fp16_c2", 2, (5, 3, 480, 640), "float16", None),
    ("autocast16", 19, (2, 3, 256, 320), "float32", "float16"),
]
PK_PPM = 15


def main(out, dsconv=False, ppm=False):
    cases, pk = (DS_CASES, PK_DSCONV) if dsconv else ((PPM_CASES, PK_PPM) if ppm else (CASES, PK_STEM))
    import numpy as np
    import torch
    import _fscnn_boot
    _fscnn_boot.load()
    from fast_scnn_pytorch_amd import _lib, arch, portable_init
    from models.fast_scnn import FastSCNN
    lib = _lib.load()
    dev = torch.device("cuda", 0)
    res = {}
    for i, (name, nc, shape, xdt, ac) in enumerate(cases):
        sd = {k: torch.from_numpy(np.asarray(v)) for k, v in
              arch.portable_state_dict(nc, seed=1, variant="bnrand").items()}
        m = FastSCNN(nc)
        m.load_state_dict(sd)
        m = m.to(dev).eval()
        m._keep_ws = bool(os.environ.get("STEM_DEBUG"))
        x = torch.from_numpy(portable_init.input_tensor(7 + i, shape)).to(dev).to(getattr(torch, xdt))
        if i == 0:
            _lib.check(lib.fscnn_prof_begin(pk, 64), "fscnn_prof_begin")
        with torch.no_grad():
            if ac:
                with torch.autocast("cuda", dtype=getattr(torch, ac)):
                    y = m(x)[0]
            else:
                y = m(x)[0]
        torch.cuda.synchronize()
        if i == 0:
            ms, n, b, f = ctypes.c_double(), ctypes.c_longlong(), ctypes.c_double(), ctypes.c_double()
            _lib.check(lib.fscnn_prof_end(ctypes.byref(ms), ctypes.byref(n), ctypes.byref(b),
                                          ctypes.byref(f)), "fscnn_prof_end")
            res["stem_launches"] = np.int64(n.value)
        res[name] = y.float().cpu().numpy()
        if os.environ.get("STEM_DEBUG") and i == 0:  # stage buffers of the first case
            for u in ("l1pw.a", "l2dw.a", "l2pw.a", "po.a", "f", "c2pw.a"):
                try:
                    res["dbg." + u] = m.debug_buffer(u).float().cpu().numpy()
                except Exception as e:  # noqa: BLE001
                    print("no buffer", u, e)
    np.savez(out, **res)


if __name__ == "__main__":
    main(sys.argv[1], "--dsconv" in sys.argv[2:], "--ppm" in sys.argv[2:])
