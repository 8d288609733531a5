"""GPU input path against the oracle restatements of
ToTensor + Normalize (train.py:104-107) and CitySegmentation._class_to_index
(data_loader/cityscapes.py:56-71): bit-exact."""
import numpy as np
import pytest
import torch

from oracle import fast_scnn_ref as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.mark.parametrize("shape", [(2, 64, 96), (1, 67, 92), (3, 1024, 2048)])
def test_normalize_images_bit_exact(shape):
    from fast_scnn_pytorch_amd.data import IMAGENET_MEAN, IMAGENET_STD, normalize_images
    rng = np.random.default_rng(11)
    imgs = rng.integers(0, 256, shape + (3,), dtype=np.uint8)
    got = normalize_images(torch.from_numpy(imgs).to(DEV)).cpu()
    for n in range(0, shape[0], max(1, shape[0] - 1)):
        want = ref.to_tensor_normalize(imgs[n], IMAGENET_MEAN, IMAGENET_STD)
        assert torch.equal(got[n], want)
    bf = normalize_images(torch.from_numpy(imgs).to(DEV), dtype=torch.bfloat16).cpu()
    assert torch.equal(bf, got.to(torch.bfloat16))


def test_normalize_feeds_the_model():
    from fast_scnn_pytorch_amd.data import normalize_images
    from models.fast_scnn import FastSCNN
    m = FastSCNN(19).to(DEV).eval()
    imgs = torch.randint(0, 256, (2, 96, 128, 3), dtype=torch.uint8, device=DEV)
    with torch.no_grad():
        out = m(normalize_images(imgs))[0]
    assert out.shape == (2, 19, 96, 128) and torch.isfinite(out).all()


def test_cityscapes_label_map():
    from fast_scnn_pytorch_amd.data import CityscapesLabelMap
    rng = np.random.default_rng(12)
    mask = rng.integers(0, 34, (2, 77, 130)).astype(np.uint8)
    got = CityscapesLabelMap()(torch.from_numpy(mask).to(DEV)).cpu().numpy()
    np.testing.assert_array_equal(got, ref.cityscapes_class_to_index(mask))
    # ids beyond the table (e.g. 255) fail like the reference's assert (cityscapes.py:66-68) ...
    bad = torch.tensor([255, 7, 33], dtype=torch.uint8, device=DEV)
    with pytest.raises(AssertionError):
        CityscapesLabelMap()(bad)
    # ... or, with strict=False, are mapped to the ignore label
    out = CityscapesLabelMap(strict=False)(bad).cpu()
    assert out.tolist() == [-1, 0, 18]
