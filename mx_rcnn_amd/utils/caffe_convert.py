"""Caffe Fast R-CNN weight conversion (reference `utils/caffe_convert.py:14-60`, which needs a
caffe build and is broken as shipped: missing symbol import, ``os.path.join(None, ...)``).

Reads a binary ``.caffemodel`` directly -- a minimal protobuf wire-format decoder of the parts
of caffe.proto the conversion needs, so neither caffe nor generated protobuf classes are
required:

  NetParameter      1 name, 100 layer (LayerParameter), 2 layers (V1LayerParameter, old nets)
  LayerParameter    1 name, 2 type (string), 7 blobs (BlobProto)
  V1LayerParameter  4 name, 5 type (enum: 4 CONVOLUTION, 14 INNER_PRODUCT), 6 blobs
  BlobProto         1 num, 2 channels, 3 height, 4 width, 5 data (float, packed or not),
                    7 shape (BlobShape: 1 dim, int64), 8 double_data

As in the reference, every Convolution / InnerProduct layer with a (weight, bias) blob pair is
converted, the first convolution's input channels are swapped BGR -> RGB, layer names have '/'
replaced by '_', weights are reshaped to the target network's argument shapes (layers the
network does not have are skipped), and the output is an MXNet-layout ``.params`` checkpoint.
An ``.npz`` export of the blobs (``<layer>_0`` = weight, ``<layer>_1`` = bias) is accepted too.
"""
import logging

import numpy as np

from .load_model import save_checkpoint

_CONV_TYPES = ('Convolution', 'InnerProduct', 4, 14)


# ------------------------------------------------------------------ protobuf wire format
def _varint(buf, i):
    shift = result = 0
    while True:
        b = buf[i]
        i += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, i
        shift += 7


def _fields(buf):
    """Yield (field_number, wire_type, value) of one message; value is an int (varint), bytes
    (length-delimited) or the raw 4 / 8 bytes (fixed32 / fixed64)."""
    i, n = 0, len(buf)
    while i < n:
        key, i = _varint(buf, i)
        fno, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 2:
            ln, i = _varint(buf, i)
            v = buf[i:i + ln]
            i += ln
        elif wt == 5:
            v = buf[i:i + 4]
            i += 4
        elif wt == 1:
            v = buf[i:i + 8]
            i += 8
        else:
            raise ValueError('unsupported protobuf wire type %d (field %d)' % (wt, fno))
        yield fno, wt, v


def _packed_varints(v):
    out, i = [], 0
    while i < len(v):
        x, i = _varint(v, i)
        out.append(x)
    return out


def parse_blob(buf):
    """BlobProto -> float32 ndarray shaped by ``shape`` (or the legacy num/channels/height/width)."""
    legacy = {}
    dims = []
    chunks, dchunks = [], []
    for fno, wt, v in _fields(buf):
        if fno in (1, 2, 3, 4) and wt == 0:
            legacy[fno] = v
        elif fno == 5:  # float data
            chunks.append(np.frombuffer(bytes(v), dtype='<f4'))  # packed (wt 2) or one fixed32 (wt 5)
        elif fno == 8:  # double data
            dchunks.append(np.frombuffer(bytes(v), dtype='<f8'))
        elif fno == 7 and wt == 2:  # BlobShape
            for f2, w2, v2 in _fields(v):
                if f2 == 1:
                    dims.extend(_packed_varints(v2) if w2 == 2 else [v2])
    if chunks:
        data = np.concatenate(chunks).astype(np.float32)
    elif dchunks:
        data = np.concatenate(dchunks).astype(np.float32)
    else:
        data = np.zeros(0, np.float32)
    if not dims:
        dims = [legacy.get(k, 1) for k in (1, 2, 3, 4)]
    return data.reshape([int(d) for d in dims]) if data.size == int(np.prod(dims)) else data


def read_caffemodel(path):
    """-> list of (layer_name, layer_type, [blob ndarrays]) in network order."""
    with open(path, 'rb') as f:
        buf = memoryview(f.read())
    layers = []
    for fno, wt, v in _fields(buf):
        if fno not in (100, 2) or wt != 2:
            continue
        v1 = fno == 2
        name, typ, blobs = '', None, []
        for f2, w2, v2 in _fields(v):
            if f2 == (4 if v1 else 1) and w2 == 2:
                name = bytes(v2).decode('utf-8')
            elif f2 == (5 if v1 else 2):
                typ = v2 if v1 else bytes(v2).decode('utf-8')
            elif f2 == (6 if v1 else 7) and w2 == 2:
                blobs.append(parse_blob(v2))
        layers.append((name, typ, blobs))
    return layers


# ------------------------------------------------------------------ encoder (tests, exports)
def _key(fno, wt):
    return _enc_varint((fno << 3) | wt)


def _enc_varint(x):
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _ld(fno, payload):
    return _key(fno, 2) + _enc_varint(len(payload)) + payload


def encode_blob(arr, legacy=False):
    arr = np.ascontiguousarray(arr, dtype='<f4')
    if legacy:
        d = list(arr.shape) + [1] * (4 - arr.ndim)
        head = b''.join(_key(k, 0) + _enc_varint(int(v)) for k, v in zip((1, 2, 3, 4), d))
    else:
        head = _ld(7, _ld(1, b''.join(_enc_varint(int(s)) for s in arr.shape)))
    return head + _ld(5, arr.tobytes())


def write_caffemodel(path, layers, v1=False):
    """layers: [(name, type, [arrays])]; ``v1`` writes the old ``layers`` / enum-type format."""
    out = bytearray(_ld(1, b'net'))
    for name, typ, blobs in layers:
        if v1:
            body = _ld(4, name.encode()) + _key(5, 0) + _enc_varint(int(typ))
            body += b''.join(_ld(6, encode_blob(b, legacy=True)) for b in blobs)
            out += _ld(2, body)
        else:
            body = _ld(1, name.encode()) + _ld(2, typ.encode())
            body += b''.join(_ld(7, encode_blob(b)) for b in blobs)
            out += _ld(100, body)
    with open(path, 'wb') as f:
        f.write(bytes(out))


# ------------------------------------------------------------------ conversion
def convert_layers(layers, arg_shapes=None):
    """(name, type, blobs) list -> {arg_name: float32 array}; the reference's rules."""
    arg = {}
    first_conv = True
    for name, typ, blobs in layers:
        if typ not in _CONV_TYPES:
            continue
        if len(blobs) != 2:
            raise ValueError('layer %s: expected (weight, bias) blobs, got %d' % (name, len(blobs)))
        name = name.replace('/', '_')
        w = np.array(blobs[0], dtype=np.float32)
        b = np.array(blobs[1], dtype=np.float32).reshape(-1)
        if first_conv and w.ndim == 4 and w.shape[1] == 3:
            w = w[:, ::-1, :, :].copy()  # BGR (caffe) -> RGB
        wname, bname = name + '_weight', name + '_bias'
        if arg_shapes is not None:
            if wname not in arg_shapes:
                logging.info('%s not in the target network, skipped', wname)
                continue
            w = w.reshape(arg_shapes[wname])
            b = b.reshape(arg_shapes[bname])
        arg[wname], arg[bname] = w, b
        if first_conv and typ in ('Convolution', 4):
            first_conv = False
    return arg


def vgg_test_arg_shapes(num_classes=21):
    """Argument shapes of the VGG16 Fast R-CNN test network (``rcnn/symbol.py``: get_vgg_test)."""
    from ..models.faster_rcnn import FasterRCNN
    return dict(FasterRCNN('vgg16', num_classes).arg_shapes('rcnn'))


def load_model(model_path, prefix_out=None, epoch_out=0, arg_shapes=None):
    """Convert a ``.caffemodel`` (or an ``.npz`` blob export) to MXNet-layout arg params and,
    with ``prefix_out``, save ``<prefix_out>-<epoch>.params``."""
    if str(model_path).endswith('.npz'):
        z = np.load(model_path, allow_pickle=False)
        per = {}
        for key in z.files:
            layer, idx = key.rsplit('_', 1)
            per.setdefault(layer, {})[int(idx)] = z[key]
        layers = [(k, 'Convolution' if v[0].ndim == 4 else 'InnerProduct', [v[0], v[1]]) for k, v in per.items()]
        # npz key order is the export order; conv1_1 must come first for the BGR swap
        layers.sort(key=lambda t: 0 if t[0] == 'conv1_1' else 1)
    else:
        layers = read_caffemodel(model_path)
    arg = convert_layers(layers, arg_shapes)
    if prefix_out is not None:
        save_checkpoint(prefix_out, epoch_out, arg, {})
    return arg
