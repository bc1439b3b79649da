"""Pickle-free roidb / proposal caches (.npz, loaded with allow_pickle=False).

The reference caches roidbs and the RPN proposal hand-off as cPickle files
(`helper/dataset/pascal_voc.py:87-99`, `rcnn/rpn/generate.py:70-76`); this framework
writes its own caches as plain arrays, so loading a cache executes nothing from the file.
"""
import os

import numpy as np
import scipy.sparse


def save_roidb(path, roidb):
    arrays = {'n': np.array([len(roidb)], np.int64)}
    for i, e in enumerate(roidb):
        arrays['%d/boxes' % i] = np.asarray(e['boxes'])
        arrays['%d/gt_classes' % i] = np.asarray(e['gt_classes'])
        ov = e['gt_overlaps']
        ov = ov.tocoo() if scipy.sparse.issparse(ov) else scipy.sparse.coo_matrix(np.asarray(ov))
        arrays['%d/ov_shape' % i] = np.array(ov.shape, np.int64)
        arrays['%d/ov_row' % i] = ov.row.astype(np.int32)
        arrays['%d/ov_col' % i] = ov.col.astype(np.int32)
        arrays['%d/ov_val' % i] = ov.data.astype(np.float32)
        arrays['%d/flipped' % i] = np.array([bool(e.get('flipped', False))])
    tmp = path + '.tmp.npz'
    np.savez(tmp, **arrays)
    os.replace(tmp, path)


def load_roidb(path):
    z = np.load(path, allow_pickle=False)
    out = []
    for i in range(int(z['n'][0])):
        shape = tuple(int(v) for v in z['%d/ov_shape' % i])
        ov = scipy.sparse.csr_matrix((z['%d/ov_val' % i], (z['%d/ov_row' % i], z['%d/ov_col' % i])), shape=shape)
        out.append({'boxes': z['%d/boxes' % i], 'gt_classes': z['%d/gt_classes' % i], 'gt_overlaps': ov,
                    'flipped': bool(z['%d/flipped' % i][0])})
    return out


def save_box_list(path, box_list):
    """RPN proposal dump: list (per image) of (n, 4) or (n, 5) arrays."""
    tmp = '%s.tmp%d.npz' % (path, os.getpid())  # write-then-rename (other ranks may read it next)
    np.savez(tmp, n=np.array([len(box_list)]), **{'b%d' % i: np.asarray(b, np.float32) for i, b in enumerate(box_list)})
    os.replace(tmp, path)


def load_box_list(path):
    z = np.load(path, allow_pickle=False)
    return [z['b%d' % i] for i in range(int(z['n'][0]))]
