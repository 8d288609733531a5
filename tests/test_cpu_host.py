"""CPU-side checks of the boundary: the C-ABI library loads, exports every symbol declared in
include/fastscnn.h, and its layer table / arena layout / plans agree with the reference schema.
No compute call is made (there is no GPU here)."""
import os
import re
import subprocess

import pytest
import torch

from fast_scnn_pytorch_amd import _lib, arch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "fastscnn.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(fscnn_\w+)\s*\(", src)))


def test_library_exports_header_symbols():
    lib = _lib.load()
    syms = header_symbols()
    assert len(syms) >= 30
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (fscnn_\w+)", out))
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    for s in syms:
        assert hasattr(lib, s)
    assert set(_lib.SIGNATURES) <= set(syms)
    assert b"gfx950" in lib.fscnn_version()


def test_code_objects_target_gfx950():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert b"gfx942" not in blob and b"sm_" not in blob.split(b"amdgcn")[0][:0]


@pytest.mark.parametrize("nc,aux", [(19, False), (2, False), (19, True)])
def test_native_table_matches_schema(nc, aux):
    from fast_scnn_pytorch_amd.fast_scnn import _Native
    nat = _Native(nc, aux)
    specs = arch.param_specs(nc, aux)
    assert [p[0] for p in nat.params] == [s[0] for s in specs]
    for (name, off, numel), (_, shape, _, _) in zip(nat.params, specs):
        n = 1
        for s in shape:
            n *= s
        assert numel == n and off % 16 == 0, name
    ends = [off + numel for _, off, numel in nat.params]
    assert max(ends) <= nat.p_total
    bufs = [b[0] for b in nat.buffers]
    assert bufs == [b[0] for b in arch.buffer_specs(nc, aux)]
    assert nat.n_bn == (45 if aux else 44)
    # backward stages tile the arena: [0, p_total)
    rs = sorted(nat.stage_ranges)
    assert rs[0][0] == 0 and rs[-1][1] == nat.p_total
    for (a, b), (c, d) in zip(rs, rs[1:]):
        assert b == c


def test_plans_and_workspace_sizes():
    from fast_scnn_pytorch_amd.fast_scnn import _Native
    nat = _Native(19, False)
    p, fw, bw = nat.plan(8, 1024, 2048, _lib.DT_BF16, True)
    assert fw > 0 and bw > 0
    dims = (_lib.c_int * 10)()
    _lib.check(nat.lib.fscnn_plan_shapes(p, dims))
    assert list(dims) == [511, 1023, 256, 512, 128, 256, 64, 128, 32, 64]
    # everything fits comfortably in one MI355X (288 GB)
    assert fw + bw < 64 * 2 ** 30
    p2, fw2, bw2 = nat.plan(1, 768, 768, _lib.DT_F32, False)
    assert bw2 == 0 and fw2 > 0
    dims2 = (_lib.c_int * 10)()
    _lib.check(nat.lib.fscnn_plan_shapes(p2, dims2))
    assert list(dims2) == [383, 383, 192, 192, 96, 96, 48, 48, 24, 24]
    # the aux head (models/fast_scnn.py:24-31) plans its im2col columns and buffers on top
    nat_aux = _Native(19, True)
    _, fwa, bwa = nat_aux.plan(2, 128, 256, _lib.DT_F32, True)
    _, fw0, bw0 = nat.plan(2, 128, 256, _lib.DT_F32, True)
    assert fwa > fw0 and bwa > bw0
    with pytest.raises(RuntimeError):
        nat.plan(0, 128, 256, _lib.DT_F32, False)


def test_module_tree_and_arena_on_cpu():
    from models.fast_scnn import FastSCNN, get_fast_scnn
    m = get_fast_scnn("citys")
    assert m.classifier.conv[1].out_channels == 19
    assert isinstance(m.global_feature_extractor.ppm.conv1.conv[0], torch.nn.Conv2d)
    sd = m.state_dict()
    assert list(sd.keys()) == list(arch.state_dict_specs(19).keys())
    ar = m.arena()  # packing only touches host tensors here
    params = list(m.parameters())
    assert all(p.untyped_storage().data_ptr() == ar["P"].untyped_storage().data_ptr()
               for p in params)
    # load_state_dict writes through the arena views
    sd2 = {k: (v + 1 if v.is_floating_point() else v) for k, v in sd.items()}
    m.load_state_dict(sd2)
    assert torch.equal(m.state_dict()["classifier.conv.1.bias"], sd["classifier.conv.1.bias"] + 1)
    assert m.arena()["P"].data_ptr() == ar["P"].data_ptr()
    with pytest.raises(RuntimeError):
        m(torch.zeros(2, 3, 64, 64))
    with pytest.raises(TypeError):
        get_fast_scnn("tusimple", num_classes=2)  # reference behaviour (duplicate argument)
    assert FastSCNN(2).classifier.conv[1].out_channels == 2


def test_pretrained_checkpoint_with_module_prefix(tmp_path):
    """train.py:449 saves the DataParallel-wrapped state_dict ('module.' keys); get_fast_scnn
    (pretrained=True) loads it into the bare model."""
    from models.fast_scnn import get_fast_scnn
    src = get_fast_scnn("tusimple")
    with torch.no_grad():
        for p in src.parameters():
            p.add_(0.5)
    sd = {"module." + k: v for k, v in src.state_dict().items()}
    torch.save(sd, str(tmp_path / "fast_scnn_tusimple.pth"))
    m = get_fast_scnn("tusimple", pretrained=True, root=str(tmp_path), map_cpu=True)
    for (k, a), (_, b) in zip(m.state_dict().items(), src.state_dict().items()):
        assert torch.equal(a, b), k


def test_fused_sgd_runs_split_at_foreign_tensors():
    """FusedSGD launches one fused kernel per run of tensors that tile a span with nothing but
    64-B alignment padding between them; a frozen / other-group tensor in between splits it."""
    from fast_scnn_pytorch_amd.optim import _runs
    # contiguous 16-float aligned tensors: [0,10) [16,40) [48,48+16)
    assert _runs([0, 16, 48], [10, 24, 16]) == [(0, 64)]
    # a foreign tensor occupies [16, 40): runs split around it
    assert _runs([0, 48], [10, 16]) == [(0, 10), (48, 64)]
    # order-independent
    assert _runs([48, 0, 16], [16, 10, 24]) == [(0, 64)]
