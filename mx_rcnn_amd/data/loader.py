"""Data iterators (reference `rcnn/loader.py:9-330`): ``AnchorLoader`` for RPN / end-to-end
training, ``ROIIter`` for Fast R-CNN on precomputed proposals and for testing.

MI355X-first differences from the reference's single-threaded MXNet DataIter:

* Anchor targets are NOT computed here: the loader ships images + gt boxes and the model
  step assigns anchors on the device (HIP kernels), so the host never runs the IoU loop.
* A background thread pool decodes / resizes the next batches while the GPU trains
  (``prefetch`` batches in flight) into pinned host memory; the trainer copies them with
  non_blocking H2D transfers.
* Data parallel: one process per GPU; every rank draws the SAME shuffled order (seeded per
  epoch) and cuts the same GLOBAL batches (``batch_size`` x world images); rank r takes its
  slice, equal by default or proportional to ``work_load_list`` (MXNet's
  ``_split_input_slice``, reference `rcnn/loader.py:114-120`).
* Shapes: like the reference's AnchorLoader, which pads every device's image to the common
  shape of the step (`rcnn/loader.py:283-286`), every rank pads its batch to the max resized
  shape over the WHOLE global batch -- computed from roidb metadata, identical on every rank
  with no communication -- and the gt count to the global max.  Both are rounded up to
  buckets (``shape_bucket`` px, power-of-two gt counts) so a dataset produces few distinct
  shapes and each gets one hipGraph; all ranks capture on the same step.  ``pad_shape`` /
  ``max_gt`` fix them outright.  The per-image scale choice is drawn from a per-(epoch,
  global batch) seed, so every rank knows every image's resized size.
* Multiple images per device are supported (the reference asserts one).
"""
import queue
import threading

import numpy as np
import torch

from ..config import config
from ..processing.image_processing import tensor_vstack
from . import minibatch


class _Prefetcher:
    def __init__(self, make_batch, n_batches, prefetch=2, workers=2):
        self.make_batch = make_batch
        self.n = n_batches
        self.q = queue.Queue(maxsize=max(1, prefetch))
        self.workers = max(1, workers)
        self._next = 0
        self._lock = threading.Lock()
        self._results = {}
        self._cv = threading.Condition()
        self._stop = False
        self._threads = [threading.Thread(target=self._work, daemon=True) for _ in range(self.workers)]
        self._sem = threading.Semaphore(max(1, prefetch) + self.workers)
        for t in self._threads:
            t.start()

    def _work(self):
        while True:
            self._sem.acquire()
            with self._lock:
                if self._stop or self._next >= self.n:
                    self._sem.release()
                    return
                i = self._next
                self._next += 1
            try:
                res = self.make_batch(i)
            except Exception as e:  # surfaced to the consumer
                res = e
            with self._cv:
                self._results[i] = res
                self._cv.notify_all()

    def get(self, i):
        with self._cv:
            while i not in self._results:
                self._cv.wait()
            res = self._results.pop(i)
        self._sem.release()
        if isinstance(res, Exception):
            raise res
        return res

    def close(self):
        with self._lock:
            self._stop = True
        for _ in self._threads:
            self._sem.release()
        for t in self._threads:
            t.join()


def _pin(t):
    t = torch.as_tensor(t)
    try:
        return t.pin_memory() if torch.cuda.is_available() else t
    except RuntimeError:
        return t


def aspect_grouped_order(roidb, rng):
    """Horizontal vs vertical groups, shuffled pairs (reference `rcnn/loader.py:62-83`)."""
    widths = np.array([r.get('width', 1) for r in roidb])
    heights = np.array([r.get('height', 1) for r in roidb])
    horz = widths >= heights
    inds = np.hstack((rng.permutation(np.where(horz)[0]), rng.permutation(np.where(~horz)[0])))
    if inds.shape[0] % 2:
        pairs = inds[:-1].reshape(-1, 2)
        inds[:-1] = pairs[rng.permutation(pairs.shape[0])].reshape(-1)
    else:
        pairs = inds.reshape(-1, 2)
        inds = pairs[rng.permutation(pairs.shape[0])].reshape(-1)
    return inds


def split_input_slice(batch_size, work_load_list):
    """Split ``batch_size`` items over devices proportionally to ``work_load_list`` ->
    list of (start, stop); every slice must be non-empty (MXNet ``_split_input_slice``)."""
    total = float(sum(work_load_list))
    counts = [int(round(w * batch_size / total)) for w in work_load_list]
    diff = batch_size - sum(counts)
    counts[-1] += diff
    if any(c <= 0 for c in counts):
        raise ValueError('work_load_list %s leaves a device without data at batch size %d'
                         % (list(work_load_list), batch_size))
    out, start = [], 0
    for c in counts:
        out.append((start, start + c))
        start += c
    return out


def _parse_work_load(wl, world):
    if wl is None:
        return None
    if isinstance(wl, str):
        wl = [float(v) for v in wl.strip('[]() ').split(',') if v.strip()]
    wl = [float(v) for v in wl]
    if len(wl) != world:
        raise ValueError('work_load_list has %d entries for %d ranks' % (len(wl), world))
    return wl


def _bucket_up(v, q):
    return int(-(-v // q) * q) if q and q > 1 else int(v)


def _pow2_at_least(n, lo=8):
    p = lo
    while p < n:
        p *= 2
    return p


class _BaseLoader:
    def __init__(self, roidb, batch_size, shuffle, mode, ctx, work_load_list, rank, world_size, seed, prefetch,
                 workers):
        self.roidb = roidb
        self.batch_size = batch_size
        self.shuffle = shuffle
        self.mode = mode
        self.ctx = ctx
        self.work_load_list = _parse_work_load(work_load_list, world_size)
        self.rank, self.world_size = rank, world_size
        self.seed = seed
        self.epoch = 0
        self.prefetch, self.workers = prefetch, workers
        self.size = len(roidb)
        self.index = np.arange(self.size)
        self.cur = 0
        self._pf = None
        self.reset()

    # -- order / sharding
    def reset(self):
        self.cur = 0
        if self._pf is not None:
            self._pf.close()
        if self.shuffle:
            rng = np.random.RandomState(self.seed + self.epoch)
            if config.TRAIN.ASPECT_GROUPING and 'width' in self.roidb[0]:
                self.index = aspect_grouped_order(self.roidb, rng)
            else:
                self.index = rng.permutation(self.size)
        self.epoch += 1
        self._batches = self._shard_batches()
        self._pf = None  # started lazily by the first __next__ of the epoch

    def close(self):
        """Stop the prefetch workers (call before exiting mid-epoch)."""
        if self._pf is not None:
            self._pf.close()
            self._pf = None

    def _shard_batches(self):
        """This rank's slice of every global batch (equal steps on every rank); the global
        batches themselves are kept for the shape plan."""
        gb = self.batch_size * self.world_size
        nb = self.size // gb
        self._global = [self.index[i * gb:(i + 1) * gb] for i in range(nb)]
        if self.work_load_list is not None and self.world_size > 1:
            a, b = split_input_slice(gb, self.work_load_list)[self.rank]
        else:
            a, b = self.rank * self.batch_size, (self.rank + 1) * self.batch_size
        self._slice = (a, b)
        return [g[a:b] for g in self._global]

    def plan_hw(self, i):
        """(pad (H, W), this rank's scale indexes) for global batch ``i``: the max resized
        shape over the global batch rounded up to ``shape_bucket`` (or ``pad_shape``)."""
        sidx = self._scale_indexes(i)
        a, b = self._slice
        if getattr(self, 'pad_shape', None) is not None:
            return tuple(self.pad_shape), sidx[a:b]
        hs, ws = [], []
        for j, si in zip(self._global[i], sidx):
            h, w = _planned_hw(self.roidb[j], config.SCALES[si])
            hs.append(h)
            ws.append(w)
        q = getattr(self, 'shape_bucket', 1)
        return (_bucket_up(max(hs), q), _bucket_up(max(ws), q)), sidx[a:b]

    def _scale_indexes(self, i):
        """Per-image SCALES choice for global batch ``i`` (same on every rank)."""
        n = len(self._global[i])
        if len(config.SCALES) == 1:
            return np.zeros(n, np.int64)
        rng = np.random.RandomState((self.seed * 1000003 + self.epoch * 7919 + i) % (2 ** 31))
        return rng.randint(0, len(config.SCALES), size=n)

    def __len__(self):
        return len(self._batches)

    @property
    def global_batch_size(self):
        """Images per step over all ranks (the Speedometer's batch size)."""
        return self.batch_size * self.world_size

    def iter_next(self):
        return self.cur < len(self._batches)

    def getindex(self):
        return self.cur

    def getpad(self):
        return 0

    def __iter__(self):
        return self

    def __next__(self):
        if not self.iter_next():
            raise StopIteration
        if self._pf is None:
            self._pf = _Prefetcher(self._make_batch, len(self._batches), self.prefetch, self.workers)
        b = self._pf.get(self.cur)
        self.cur += 1
        return b

    next = __next__

    def get_batch(self):
        if not self._batches:
            raise ValueError('%d images do not fill one global batch of %d (%d per rank x %d ranks)'
                             % (self.size, self.batch_size * self.world_size, self.batch_size, self.world_size))
        return self._make_batch(min(self.cur, len(self._batches) - 1))


class AnchorLoader(_BaseLoader):
    """RPN / end-to-end loader.  Batches: data (B,3,H,W) fp32, im_info (B,3), gt_boxes (B,G,5)
    padded with -1, n_gt (B,) int32.  ``feat_sym`` (the model, or anything with
    ``feat_shape(h, w)``) is kept for API parity and shape reporting."""

    def __init__(self, feat_sym, roidb, batch_size=1, shuffle=False, mode='train', ctx=None, work_load_list=None,
                 feat_stride=16, anchor_scales=(8, 16, 32), anchor_ratios=(0.5, 1, 2), allowed_border=0,
                 need_mean=True, rank=0, world_size=1, seed=0, prefetch=2, workers=2, pad_shape=None, max_gt=None,
                 shape_bucket=None, raw_images=False):
        self.feat_sym = feat_sym
        self.raw_images = raw_images
        self.feat_stride, self.anchor_scales, self.anchor_ratios = feat_stride, anchor_scales, anchor_ratios
        self.allowed_border, self.need_mean = allowed_border, need_mean
        self.pad_shape, self.max_gt = pad_shape, max_gt
        # shape bucketing only pays when shapes are static per bucket (graph replay); with a single
        # process and no bucket requested, pad to the batch max like the reference's tensor_vstack
        self.shape_bucket = shape_bucket if shape_bucket is not None else (64 if world_size > 1 else 1)
        self.data_name = ['data', 'im_info']
        self.label_name = ['gt_boxes', 'n_gt']
        super().__init__(roidb, batch_size, shuffle, mode, ctx, work_load_list, rank, world_size, seed, prefetch,
                         workers)

    def step_plan(self, i):
        """(pad_hw, gt_slots, scale_indexes of this rank's images) for global batch ``i``; the
        same (pad_hw, gt_slots) on every rank."""
        hw, sidx = self.plan_hw(i)
        glob = [self.roidb[j] for j in self._global[i]]
        if self.max_gt is not None:
            G = self.max_gt
        else:
            # power-of-two gt slots (n_gt carries the count): a handful of input shapes, so the
            # per-shape hipGraph cache does not capture a graph for every distinct gt count
            G = _pow2_at_least(max(1, max(int((e['gt_classes'] != 0).sum()) for e in glob)))
        return hw, G, sidx

    def _make_batch(self, i):
        entries = [self.roidb[j] for j in self._batches[i]]
        (ph, pw), G, sidx = self.step_plan(i)
        data, label = minibatch.get_minibatch(entries, 0, self.mode, need_mean=self.need_mean, has_rpn=True,
                                              scale_indexes=sidx, raw=self.raw_images)
        im = data['data']
        if self.raw_images:
            return self._raw_batch(im, data['im_info'], (ph, pw), label, G, len(entries))
        if im.shape[2] > ph or im.shape[3] > pw:
            raise ValueError('image %s larger than the planned pad shape %s' % (im.shape[2:], (ph, pw)))
        if im.shape[2] != ph or im.shape[3] != pw:
            padded = np.zeros((im.shape[0], 3, ph, pw), np.float32)
            padded[:, :, :im.shape[2], :im.shape[3]] = im
            im = padded
        gts = label.get('gt_boxes', [np.zeros((0, 5), np.float32)] * len(entries))
        gt = np.full((len(entries), G, 5), -1.0, np.float32)
        n_gt = np.zeros((len(entries),), np.int32)
        for k, g in enumerate(gts):
            n = min(g.shape[0], G)
            gt[k, :n] = g[:n]
            n_gt[k] = n
        return {'data': _pin(np.ascontiguousarray(im, dtype=np.float32)), 'im_info': _pin(data['im_info']),
                'gt_boxes': _pin(gt), 'n_gt': _pin(n_gt)}

    def _raw_batch(self, im, im_info, hw, label, G, n):
        """raw_images: uint8 (B, ph, pw, 3) BGR, zero padded; the device converts it (ops/image.py)
        with ``pixel_means`` (zeros when the network does not subtract them)."""
        ph, pw = hw
        if im.shape[1] > ph or im.shape[2] > pw:
            raise ValueError('image %s larger than the planned pad shape %s' % (im.shape[1:3], hw))
        if im.shape[1] != ph or im.shape[2] != pw:
            padded = np.zeros((im.shape[0], ph, pw, 3), np.uint8)
            padded[:, :im.shape[1], :im.shape[2]] = im
            im = padded
        gts = label.get('gt_boxes', [np.zeros((0, 5), np.float32)] * n)
        gt = np.full((n, G, 5), -1.0, np.float32)
        n_gt = np.zeros((n,), np.int32)
        for k, g in enumerate(gts):
            m = min(g.shape[0], G)
            gt[k, :m] = g[:m]
            n_gt[k] = m
        means = np.asarray(config.PIXEL_MEANS, np.float64).reshape(-1)[:3] if self.need_mean else np.zeros(3)
        return {'data': _pin(im), 'im_info': _pin(im_info), 'gt_boxes': _pin(gt), 'n_gt': _pin(n_gt),
                'pixel_means': torch.from_numpy(means.astype(np.float64))}

    @property
    def provide_data(self):
        b = self.get_batch()
        if self.raw_images:  # the network's input shape
            n, h, w, _ = b['data'].shape
            return [('data', (n, 3, h, w)), ('im_info', tuple(b['im_info'].shape))]
        return [('data', tuple(b['data'].shape)), ('im_info', tuple(b['im_info'].shape))]

    @property
    def provide_label(self):
        b = self.get_batch()
        out = [('gt_boxes', tuple(b['gt_boxes'].shape))]
        if self.feat_sym is not None and hasattr(self.feat_sym, 'feat_shape'):
            n, _, ih, iw = self.provide_data[0][1]
            h, w = self.feat_sym.feat_shape(ih, iw)
            A = len(self.anchor_scales) * len(self.anchor_ratios)
            out += [('label', (n, A * h * w)), ('bbox_target', (n, 4 * A, h, w)),
                    ('bbox_inside_weight', (n, 4 * A, h, w)),
                    ('bbox_outside_weight', (n, 4 * A, h, w))]
        return out


class ROIIter(_BaseLoader):
    """Fast R-CNN loader (offline proposals).  train: data, rois (B*R, 5), label, bbox_target,
    bbox_inside_weight, bbox_outside_weight; test: data, rois, im_info."""

    def __init__(self, roidb, batch_size=2, shuffle=False, mode='train', ctx=None, work_load_list=None,
                 rank=0, world_size=1, seed=0, prefetch=2, workers=2, need_mean=True, pad_shape=None,
                 shape_bucket=None):
        self.num_classes = roidb[0]['gt_overlaps'].shape[1]
        self.need_mean = need_mean
        self.pad_shape = pad_shape
        self.shape_bucket = shape_bucket if shape_bucket is not None else (64 if world_size > 1 else 1)
        self.data_name = ['data', 'rois']
        self.label_name = ['label', 'bbox_target', 'bbox_inside_weight', 'bbox_outside_weight']
        super().__init__(roidb, batch_size, shuffle, mode, ctx, work_load_list, rank, world_size, seed, prefetch,
                         workers)

    def _make_batch(self, i):
        entries = [self.roidb[j] for j in self._batches[i]]
        sidx = None
        if self.mode == 'train':
            (ph, pw), sidx = self.plan_hw(i)
        data, label = minibatch.get_minibatch(entries, self.num_classes, self.mode, need_mean=self.need_mean,
                                              has_rpn=False, scale_indexes=sidx)
        im = data['data']
        if sidx is not None and (im.shape[2] != ph or im.shape[3] != pw):
            padded = np.zeros((im.shape[0], 3, ph, pw), np.float32)
            padded[:, :, :im.shape[2], :im.shape[3]] = im
            im = padded
        out = {'data': _pin(np.ascontiguousarray(im, dtype=np.float32))}
        if self.mode == 'train':
            out['rois'] = _pin(data['rois'].reshape(-1, 5).astype(np.float32))
            out['label'] = _pin(label['label'].reshape(-1).astype(np.int32))
            for k in ('bbox_target', 'bbox_inside_weight', 'bbox_outside_weight'):
                out[k] = _pin(label[k].reshape(-1, label[k].shape[-1]).astype(np.float32))
        else:
            out['rois'] = _pin(data['rois'].astype(np.float32))
            out['im_info'] = _pin(data['im_info'])
        return out

    @property
    def provide_data(self):
        b = self.get_batch()
        return [(k, tuple(b[k].shape)) for k in ('data', 'rois')]

    @property
    def provide_label(self):
        b = self.get_batch()
        return [(k, tuple(b[k].shape)) for k in self.label_name if k in b]


def _planned_hw(entry, target_size):
    """Resized (h, w) of a roidb entry at ``target_size`` (image_processing.resize rule)."""
    from ..processing.image_processing import compute_scale
    h, w = entry.get('height'), entry.get('width')
    if h is None or w is None:
        h, w = minibatch.load_image(entry).shape[:2]
    s = compute_scale((h, w), target_size, config.MAX_SIZE)
    return int(round(h * s)), int(round(w * s))


def tensor_vstack_batches(batches, key, pad=0):
    return tensor_vstack([b[key] for b in batches], pad=pad)
