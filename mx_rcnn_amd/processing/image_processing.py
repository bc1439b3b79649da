"""Image resize / tensor conversion (reference: `helper/processing/image_processing.py:5-83`).

No OpenCV in this stack: ``imread`` uses PIL and ``resize`` uses an
align-corners=False bilinear filter without antialiasing, which is the
``cv2.INTER_LINEAR`` sampling rule (cv2 rounds uint8 math in fixed point, so
pixels may differ by 1 LSB).  Images are BGR HWC uint8 like cv2's.
"""
import numpy as np


def imread(path):
    """Read an image as BGR uint8 HWC (the cv2.imread convention)."""
    from PIL import Image
    with Image.open(path) as im:
        rgb = np.asarray(im.convert('RGB'))
    return np.ascontiguousarray(rgb[:, :, ::-1])


def imwrite(path, im_bgr):
    from PIL import Image
    Image.fromarray(np.ascontiguousarray(im_bgr[:, :, ::-1].astype(np.uint8))).save(path)


def image_size(path):
    """(height, width) without decoding pixels."""
    from PIL import Image
    with Image.open(path) as im:
        w, h = im.size
    return h, w


def compute_scale(im_shape, target_size, max_size):
    im_size_min = np.min(im_shape[0:2])
    im_size_max = np.max(im_shape[0:2])
    im_scale = float(target_size) / float(im_size_min)
    if np.round(im_scale * im_size_max) > max_size:
        im_scale = float(max_size) / float(im_size_max)
    return im_scale


def resize_bilinear(im, out_h, out_w):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(im)).permute(2, 0, 1)[None].float()
    t = torch.nn.functional.interpolate(t, size=(out_h, out_w), mode='bilinear', align_corners=False)
    out = t[0].permute(1, 2, 0).numpy()
    if im.dtype == np.uint8:
        out = np.clip(np.round(out), 0, 255).astype(np.uint8)
    return out


def resize(im, target_size, max_size):
    """Short side -> target_size, long side capped at max_size; returns (im, scale)."""
    im_scale = compute_scale(im.shape, target_size, max_size)
    out_h = int(round(im.shape[0] * im_scale))
    out_w = int(round(im.shape[1] * im_scale))
    if (out_h, out_w) == tuple(im.shape[:2]) and im_scale == 1.0:
        return im, im_scale  # the identity resample (cv2.resize returns the same pixels)
    return resize_bilinear(im, out_h, out_w), im_scale


def transform(im, pixel_means, need_mean=False):
    """BGR HWC -> RGB float (1, 3, H, W), optional mean subtraction."""
    im = im[:, :, ::-1].astype(np.float64)
    if need_mean:
        im = im - pixel_means
    return im[np.newaxis].transpose((0, 3, 1, 2))


def transform_inverse(im_tensor, pixel_means):
    assert im_tensor.shape[0] == 1
    im = im_tensor.transpose((0, 2, 3, 1))[0].copy()
    assert im.shape[2] == 3
    im += pixel_means
    return im.astype(np.uint8)


def tensor_vstack(tensor_list, pad=0):
    """Pad every dim >= 1 to the max and stack on dim 0 (1-D inputs are hstacked)."""
    ndim = len(tensor_list[0].shape)
    if ndim == 1:
        return np.hstack(tensor_list)
    dims = [max(t.shape[d] for t in tensor_list) for d in range(1, ndim)]
    out = []
    for t in tensor_list:
        pad_shape = [(0, 0)] + [(0, dims[d - 1] - t.shape[d]) for d in range(1, ndim)]
        out.append(np.pad(t, pad_shape, 'constant', constant_values=pad))
    return np.vstack(out)
