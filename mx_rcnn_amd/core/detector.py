"""Detector (reference `rcnn/detector.py:8-81`) with device-side post-processing.

The reference rebinds an executor for every image (`rcnn/detector.py:55`); here the model is
built once, weights live on the device, and an image batch runs ``model.detect``.  Optional
RoI de-duplication (TEST.DEDUP_BOXES, Fast R-CNN mode) hashes rounded RoIs like the
reference.  ``im_detect`` returns numpy (scores, pred_boxes) for API parity;
``detect_batch`` keeps everything on the device and performs the whole test-time
post-process (decode, clip, per-class score threshold, per-class NMS, top-k over classes) as
two kernel launches for the whole batch (SURVEY kernel K18, csrc/hip/det_post.hip).
"""
import numpy as np
import torch

from ..config import config
from ..ops.boxes import bbox_pred, clip_boxes
from ..ops.nms import batched_nms


DTYPES = {'fp32': torch.float32, 'bf16': torch.bfloat16, 'fp16': torch.float16}


def resolve_dtype(d):
    """'fp32' / 'bf16' / 'fp16' or a torch dtype -> torch dtype (None stays None)."""
    if d is None or isinstance(d, torch.dtype):
        return d
    if d not in DTYPES:
        raise ValueError('dtype must be one of %s, not %r' % (sorted(DTYPES), d))
    return DTYPES[d]


def _inference_copy(model, dtype):
    """A private copy of ``model`` for the test graph, its conv / FC weights in ``dtype`` (fp32:
    the masters as fp32).  The caller's model is never modified: a model still being trained can be
    evaluated between epochs, and the trainer's attachments (its filter-cache join, non-finite
    counter, dropout counter) are not copied."""
    import copy
    from ..models.layers import Conv, Linear
    held = []
    for m in model.modules():
        for k in ('pre_backward', 'nonfinite_counter', 'rng_step'):
            if m.__dict__.get(k) is not None:
                held.append((m, k, m.__dict__[k]))
                m.__dict__[k] = None
    try:
        out = copy.deepcopy(model)
    finally:
        for m, k, v in held:
            m.__dict__[k] = v
    with torch.no_grad():
        for m in out.modules():
            if isinstance(m, (Conv, Linear)):
                w = m.weight.data.to(dtype)
                m.weight.data = w.contiguous(memory_format=torch.channels_last) if w.dim() == 4 else w.contiguous()
                if m.bias is not None:
                    m.bias.data = m.bias.data.to(dtype)
            elif hasattr(m, 'moving_var'):  # BN parameters / statistics stay fp32
                for t in (m.gamma, m.beta):
                    t.data = t.data.float()
    return out.eval()


class Detector(object):
    """Test-time runner of a FasterRCNN (reference `rcnn/detector.py:8-81`).

    compute_dtype: 'fp32' / torch.float32 (the reference's precision: on the GPU every MFMA operand
    and every tensor between kernels is the exact fp32 value as three bf16 planes -- the training
    headline's fp32 mode, ops/precision.py -- on our kernels, no vendor conv / GEMM), 'bf16' (GPU
    default) or 'fp16' (BASELINE config 5's fp16 MFMA path).  On the GPU the detector runs a
    private copy of the model's weights in that precision (``self.model``); ``self.source`` is the
    model it was built from, left untouched.
    """

    def __init__(self, symbol, ctx=None, arg_params=None, aux_params=None, compute_dtype=None):
        self.ctx = torch.device(ctx) if ctx is not None else torch.device('cpu')
        if arg_params is not None or aux_params is not None:
            from .module import MutableModule
            mod = MutableModule(symbol, context=self.ctx, use_graph=False)
            mod.bind(for_training=False)
            mod.init_params(None, arg_params, aux_params, allow_missing=True)
        self.source = symbol
        compute_dtype = resolve_dtype(compute_dtype)
        if compute_dtype is None:
            compute_dtype = torch.bfloat16 if self.ctx.type == 'cuda' else torch.float32
        if compute_dtype not in (torch.bfloat16, torch.float16, torch.float32):
            raise ValueError('compute_dtype must be torch.bfloat16, torch.float16 or torch.float32 (got %s)'
                             % compute_dtype)
        self.dtype = compute_dtype
        # fp32 on the GPU: three-plane mode (MXR_FP32_EVAL=torch: plain fp32 PyTorch / vendor ops, a
        # reference arm for precision probes)
        self.planes = 3 if (self.ctx.type == 'cuda' and compute_dtype == torch.float32 and
                            __import__('os').environ.get('MXR_FP32_EVAL', 'x3') != 'torch') else 0
        if self.ctx.type == 'cuda':
            symbol.to(self.ctx)
            self.model = _inference_copy(symbol, compute_dtype)
        else:
            self.model = symbol.to(self.ctx).eval()

    def precision_scope(self):
        """Context in which this detector's model runs (the three-plane mode for GPU fp32)."""
        from ..ops.precision import x2_mode
        return x2_mode(self.planes)

    @torch.no_grad()
    def detect(self, data, im_info, rois=None):
        """model.detect of a prepared (``_prep``) batch in this detector's precision."""
        with self.precision_scope():
            return self.model.detect(data, im_info, rois)

    @torch.no_grad()
    def rpn_test(self, data, im_info):
        with self.precision_scope():
            return self.model.rpn_test(data, im_info)

    def _prep(self, im_array):
        x = torch.as_tensor(np.asarray(im_array) if not torch.is_tensor(im_array) else im_array)
        # fp32 mode: the stem kernel takes the fp32 image and writes the three planes
        x = x.to(self.ctx, self.dtype)
        if self.ctx.type == 'cuda':
            x = x.contiguous(memory_format=torch.channels_last)
        return x

    @torch.no_grad()
    def forward(self, im_array, im_info=None, roi_array=None):
        data = self._prep(im_array)
        info = None if im_info is None else torch.as_tensor(np.asarray(im_info) if not torch.is_tensor(im_info)
                                                            else im_info).float().to(self.ctx)
        rois = None if roi_array is None else torch.as_tensor(np.asarray(roi_array) if not torch.is_tensor(roi_array)
                                                              else roi_array).float().to(self.ctx)
        return self.detect(data, info, rois)

    @torch.no_grad()
    def im_detect(self, im_array, im_info=None, roi_array=None):
        """-> (scores (R, C), pred_boxes (R, 4C)) numpy, boxes in network-input pixels."""
        inv = None
        if config.TEST.DEDUP_BOXES > 0 and not config.TEST.HAS_RPN and roi_array is not None:
            v = np.array([1, 1e3, 1e6, 1e9, 1e12])
            hashes = np.round(np.asarray(roi_array) * config.TEST.DEDUP_BOXES).dot(v)
            _, index, inv = np.unique(hashes, return_index=True, return_inverse=True)
            roi_array = np.asarray(roi_array)[index, :]
        rois, scores, deltas = self.forward(im_array, im_info, roi_array)
        h, w = int(np.asarray(im_array).shape[-2] if not torch.is_tensor(im_array) else im_array.shape[-2]), \
            int(np.asarray(im_array).shape[-1] if not torch.is_tensor(im_array) else im_array.shape[-1])
        boxes = clip_boxes(bbox_pred(rois[:, 1:5].float(), deltas.float()), h, w)
        scores, boxes = scores.cpu().numpy(), boxes.cpu().numpy()
        if inv is not None:
            scores, boxes = scores[inv], boxes[inv]
        return scores, boxes

    @torch.no_grad()
    def detect_batch(self, im_array, im_info, thresh=0.05, nms_thresh=None, max_per_image=100, rois=None):
        """Batched inference + on-device post-processing.

        Returns a list (per image) of (boxes (k, 4) in ORIGINAL image pixels, scores (k,),
        classes (k,)) tensors on the device.
        """
        nms_thresh = config.TEST.NMS if nms_thresh is None else nms_thresh
        r, scores, deltas = self.forward(im_array, im_info, rois)
        info = torch.as_tensor(np.asarray(im_info) if not torch.is_tensor(im_info) else im_info).float().to(self.ctx)
        return self.postprocess(r, scores, deltas, info, nms_thresh, thresh, max_per_image)

    @staticmethod
    def device_postprocess_ok(r, scores, info):
        B = info.shape[0]
        if not (r.is_cuda and B > 0 and r.shape[0] % B == 0 and r.shape[0] // B <= 1024 and
                2 <= scores.shape[1] <= 1025):
            return False
        return True

    @torch.no_grad()
    def postprocess_raw(self, r, scores, deltas, info, nms_thresh=0.3, thresh=0.05, max_per_image=100, cap=None):
        """The whole test post-process as two device launches, no host sync (csrc/hip/det_post.hip):
        -> dets (B, cap, 6) [x1 y1 x2 y2 score class] in original-image pixels, counts (B,) int32.
        Detections are in class order, score-descending within a class."""
        from ..ops._ext import need_ext
        cap = cap or max(4 * max_per_image, 512)
        return need_ext().det_postprocess(r.float().contiguous(), scores.float().contiguous(),
                                          deltas.float().contiguous(), info.float().contiguous(), float(thresh),
                                          float(nms_thresh), int(max_per_image), int(cap))

    @torch.no_grad()
    def postprocess(self, r, scores, deltas, info, nms_thresh=0.3, thresh=0.05, max_per_image=100):
        """Device-side test post-process of ``model.detect`` outputs (see detect_batch).  GPU: the
        fused kernels plus ONE host read of the per-image counts; CPU: the tensor reference."""
        if self.device_postprocess_ok(r, scores, info):
            dets, counts = self.postprocess_raw(r, scores, deltas, info, nms_thresh, thresh, max_per_image)
            n = counts.cpu().tolist()
            return [(dets[b, :k, :4], dets[b, :k, 4], dets[b, :k, 5].long()) for b, k in enumerate(n)]
        return self.postprocess_ref(r, scores, deltas, info, nms_thresh, thresh, max_per_image)

    @torch.no_grad()
    def postprocess_ref(self, r, scores, deltas, info, nms_thresh=0.3, thresh=0.05, max_per_image=100):
        """Tensor reference of the post-process (the oracle of the device kernels)."""
        B = info.shape[0]
        C = scores.shape[1]
        out = []
        for b in range(B):
            sel = r[:, 0] == b
            rb, sb, db = r[sel], scores[sel], deltas[sel]
            boxes = clip_boxes(bbox_pred(rb[:, 1:5], db), info[b, 0], info[b, 1]).reshape(-1, C, 4)[:, 1:]
            s = sb[:, 1:]
            cls = torch.arange(1, C, device=s.device).expand_as(s)
            m = s > thresh
            bx, sc, cl = boxes[m], s[m], cls[m]
            keep = batched_nms(bx, sc, cl, nms_thresh)
            bx, sc, cl = bx[keep], sc[keep], cl[keep]
            if max_per_image > 0 and sc.numel() > max_per_image:
                th = torch.sort(sc, descending=True).values[max_per_image - 1]
                k = sc >= th
                bx, sc, cl = bx[k], sc[k], cl[k]
            out.append((bx / info[b, 2], sc, cl))
        return out
