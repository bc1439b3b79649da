"""Raw-image loader path (data/loader.py raw_images + ops/image.py): the device-side conversion
gives exactly the reference host transform's network input (BGR -> RGB, float64 minus
PIXEL_MEANS, zero pad to the batch shape: `helper/processing/image_processing.py`)."""
import numpy as np
import pytest
import torch

from mx_rcnn_amd.config import config
from mx_rcnn_amd.data.load_data import load_synthetic_roidb
from mx_rcnn_amd.data.loader import AnchorLoader
from mx_rcnn_amd.ops.image import image_prep


def _loaders(need_mean):
    _, roidb = load_synthetic_roidb(4, 90, 130, 5, flip=True, seed=3)
    # two scales so the images of a batch differ in size (padding inside the batch)
    old = (config.SCALES, config.MAX_SIZE)
    config.SCALES, config.MAX_SIZE = (90, 60), 200
    try:
        mk = lambda raw: AnchorLoader(None, roidb, batch_size=2, shuffle=True, need_mean=need_mean, seed=5,
                                      prefetch=1, workers=1, raw_images=raw)
        a, b = mk(False), mk(True)
        out = [(next(a), next(b)) for _ in range(3)]
        a.close()
        b.close()
    finally:
        config.SCALES, config.MAX_SIZE = old
    return out


@pytest.mark.parametrize('need_mean', [True, False])
def test_raw_batches_convert_to_the_host_transform(need_mean):
    for ref, raw in _loaders(need_mean):
        assert raw['data'].dtype == torch.uint8 and raw['data'].shape[-1] == 3
        assert torch.equal(raw['im_info'], ref['im_info']) and torch.equal(raw['gt_boxes'], ref['gt_boxes'])
        x = image_prep(raw['data'], raw['im_info'], raw['pixel_means'], torch.float32, channels_last=False)
        assert x.shape == ref['data'].shape
        assert torch.equal(x, ref['data']), float((x - ref['data']).abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
def test_image_prep_kernel_matches_cpu(cuda, dtype):
    g = torch.Generator().manual_seed(0)
    img = torch.randint(0, 256, (3, 61, 97, 3), generator=g, dtype=torch.uint8)
    info = torch.tensor([[61., 97., 1.], [40., 97., 1.], [61., 33., 1.]])
    means = np.asarray(config.PIXEL_MEANS)
    ref = image_prep(img, info, means, torch.float32, channels_last=False).to(dtype)
    got = image_prep(img.to(cuda), info.to(cuda), means, dtype)
    assert got.is_contiguous(memory_format=torch.channels_last) and got.dtype == dtype
    assert torch.equal(got.cpu(), ref)
