"""Caffe Fast R-CNN VGG16 weight conversion (reference `utils/caffe_convert.py`, which is
broken there: missing symbol import, ``os.path.join(None, ...)``).

Caffe / protobuf are not available in this stack, so the input is an ``.npz`` export of the
Caffe blobs (``<layer>_0`` = weight, ``<layer>_1`` = bias, as produced by any
``net.params`` dump).  conv1_1 input channels are swapped BGR -> RGB (the framework feeds RGB);
output is an MXNet-layout ``.params`` checkpoint.
"""
import numpy as np

from .load_model import save_checkpoint


def load_model(npz_path, prefix_out, epoch_out=0):
    z = np.load(npz_path, allow_pickle=False)
    arg = {}
    for key in z.files:
        layer, idx = key.rsplit('_', 1)
        arr = z[key].astype(np.float32)
        if layer == 'conv1_1' and idx == '0':
            arr = arr[:, ::-1, :, :].copy()
        arg['%s_%s' % (layer, 'weight' if idx == '0' else 'bias')] = arr
    save_checkpoint(prefix_out, epoch_out, arg, {})
    return arg
