"""MXNet NDArray-list binary codec (``mx.nd.save`` / ``mx.nd.load`` file format),
without MXNet.  Writes V2; reads V2, V1 and legacy (pre-magic) records.

File:   uint64 0x112 | uint64 0 | uint64 n | n x NDArray | uint64 n_names | n x (uint64 len, bytes)
V2:     uint32 0xF993FAC9 | int32 stype(0 = dense) | uint32 ndim | int64 dims[ndim]
        | int32 dev_type | int32 dev_id | int32 type_flag | raw little-endian data
V1:     uint32 0xF993FAC8 | uint32 ndim | uint32 dims[ndim] | ctx | type_flag | data
legacy: uint32 ndim | uint32 dims[ndim] | ctx | type_flag | data

Checkpoints are only ever parsed as data (no pickle), so loading a foreign file executes
nothing from it.  Compatibility with real MXNet-written files is unverified in this
environment (no MXNet, no fixture in the reference tree); the layout follows the spec above.
"""
import os
import struct

import numpy as np

LIST_MAGIC = 0x112
V2_MAGIC = 0xF993FAC9
V1_MAGIC = 0xF993FAC8
TYPE_FLAGS = {0: np.float32, 1: np.float64, 2: np.float16, 3: np.uint8, 4: np.int32, 5: np.int8, 6: np.int64}
FLAG_OF = {np.dtype(v): k for k, v in TYPE_FLAGS.items()}


def _to_numpy(v):
    if hasattr(v, 'detach'):
        v = v.detach().cpu()
        if str(v.dtype) == 'torch.bfloat16':
            v = v.float()
        v = v.numpy()
    return np.ascontiguousarray(np.asarray(v))


def save(fname, data):
    """Save a dict name->array (or a list of arrays) in the MXNet NDArray-list format."""
    if isinstance(data, dict):
        names = list(data.keys())
        arrays = [data[k] for k in names]
    else:
        names, arrays = [], list(data)
    # write-then-rename: a reader on another rank (alternate training loads the checkpoint the
    # previous stage wrote) never sees a partial file
    tmp = '%s.tmp%d' % (fname, os.getpid())
    with open(tmp, 'wb') as f:
        f.write(struct.pack('<QQQ', LIST_MAGIC, 0, len(arrays)))
        for a in arrays:
            a = _to_numpy(a)
            if a.dtype not in FLAG_OF:
                a = a.astype(np.float32)
            f.write(struct.pack('<IiI', V2_MAGIC, 0, a.ndim))
            if a.ndim:
                f.write(struct.pack('<%dq' % a.ndim, *a.shape))
            f.write(struct.pack('<iii', 1, 0, FLAG_OF[a.dtype]))
            f.write(a.astype(a.dtype.newbyteorder('<'), copy=False).tobytes())
        f.write(struct.pack('<Q', len(names)))
        for n in names:
            b = n.encode('utf-8')
            f.write(struct.pack('<Q', len(b)))
            f.write(b)
    os.replace(tmp, fname)


class _Reader:
    def __init__(self, buf):
        self.buf, self.pos = buf, 0

    def take(self, fmt):
        size = struct.calcsize(fmt)
        if self.pos + size > len(self.buf):
            raise ValueError('truncated NDArray file')
        out = struct.unpack_from(fmt, self.buf, self.pos)
        self.pos += size
        return out

    def raw(self, n):
        if self.pos + n > len(self.buf):
            raise ValueError('truncated NDArray file')
        out = self.buf[self.pos:self.pos + n]
        self.pos += n
        return out


def _read_array(r):
    (first,) = r.take('<I')
    if first == V2_MAGIC:
        (stype,) = r.take('<i')
        if stype != 0:
            raise ValueError('sparse NDArray (stype=%d) not supported' % stype)
        (ndim,) = r.take('<I')
        shape = r.take('<%dq' % ndim) if ndim else ()
    elif first == V1_MAGIC:
        (ndim,) = r.take('<I')
        shape = r.take('<%dI' % ndim) if ndim else ()
    else:
        ndim = first
        shape = r.take('<%dI' % ndim) if ndim else ()
    if ndim == 0:
        return np.zeros((0,), np.float32)
    r.take('<ii')  # context (dev_type, dev_id): always loaded to host
    (flag,) = r.take('<i')
    if flag not in TYPE_FLAGS:
        raise ValueError('unknown NDArray type_flag %d' % flag)
    dt = np.dtype(TYPE_FLAGS[flag]).newbyteorder('<')
    n = int(np.prod(shape))
    arr = np.frombuffer(r.raw(n * dt.itemsize), dtype=dt, count=n).reshape(shape)
    return arr.astype(dt.newbyteorder('='), copy=True)


def load(fname):
    """Load an MXNet NDArray-list file -> dict (if named) or list of numpy arrays."""
    with open(fname, 'rb') as f:
        buf = f.read()
    r = _Reader(buf)
    magic, _reserved = r.take('<QQ')
    if magic != LIST_MAGIC:
        raise ValueError('%s: not an MXNet NDArray file (magic 0x%x)' % (fname, magic))
    (n,) = r.take('<Q')
    arrays = [_read_array(r) for _ in range(n)]
    (nn,) = r.take('<Q')
    names = []
    for _ in range(nn):
        (ln,) = r.take('<Q')
        names.append(r.raw(ln).decode('utf-8'))
    if nn == 0:
        return arrays
    if nn != n:
        raise ValueError('name/array count mismatch')
    return dict(zip(names, arrays))
