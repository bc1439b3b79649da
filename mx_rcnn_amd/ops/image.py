"""Network input from raw uint8 images (csrc/hip/image.hip).

The reference's loader converts every image on the host: BGR -> RGB, float64 minus PIXEL_MEANS,
transpose to (1, 3, H, W), zero pad to the batch shape (`helper/processing/image_processing.py`
transform / tensor_vstack, `rcnn/minibatch.py` get_image_array).  At 800x1333 that host work
(~60 ms per image in numpy) and the fp32 host->device copy (12.8 MB) cap a CLI training loop far
below what the GPU step sustains.  The raw path (``AnchorLoader(raw_images=True)``) ships the
resized uint8 image instead and this op does the conversion on the device, inside the captured
step: same values bit for bit (double arithmetic, one rounding), a quarter of the copy.
"""
import numpy as np
import torch

from ._ext import need_ext


def means_of(pixel_means):
    """(3,) RGB means as python floats (config.PIXEL_MEANS, shape (1, 1, 3)), or zeros."""
    if pixel_means is None:
        return [0.0, 0.0, 0.0]
    m = np.asarray(pixel_means, dtype=np.float64).reshape(-1)
    return [float(v) for v in m[:3]]


def image_prep(img, im_info, pixel_means=None, dtype=torch.float32, channels_last=True):
    """uint8 BGR (B, H, W, 3) zero-padded images -> (B, 3, H, W) ``dtype`` RGB minus the means, 0
    outside each image's resized (h, w) = im_info[b, :2]; channels_last on the GPU."""
    means = means_of(pixel_means)
    if img.is_cuda and dtype in (torch.float32, torch.bfloat16):
        ext = need_ext()
        info = im_info if (im_info.dtype == torch.float32 and im_info.is_contiguous()) else \
            im_info.float().contiguous()
        return ext.image_prep(img.contiguous(), info, means, dtype == torch.bfloat16)
    x = img[..., [2, 1, 0]].to(torch.float64) - torch.tensor(means, dtype=torch.float64, device=img.device)
    H, W = img.shape[1], img.shape[2]
    hh = torch.arange(H, device=img.device).view(1, H, 1)
    ww = torch.arange(W, device=img.device).view(1, 1, W)
    info = im_info.to(img.device)
    valid = (hh < info[:, 0].long().view(-1, 1, 1)) & (ww < info[:, 1].long().view(-1, 1, 1))
    x = torch.where(valid[..., None], x, torch.zeros((), dtype=x.dtype, device=x.device))
    out = x.to(torch.float32).to(dtype).permute(0, 3, 1, 2)
    return out if channels_last else out.contiguous()
