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


class Detector(object):
    def __init__(self, symbol, ctx=None, arg_params=None, aux_params=None, compute_dtype=None):
        self.model = symbol
        self.ctx = torch.device(ctx) if ctx is not None else torch.device('cpu')
        if arg_params is not None or aux_params is not None:
            from .module import MutableModule
            mod = MutableModule(symbol, context=self.ctx, use_graph=False)
            mod.bind(for_training=False)
            mod.init_params(None, arg_params, aux_params, allow_missing=True)
        self.model.to(self.ctx).eval()
        if compute_dtype is None:
            compute_dtype = torch.bfloat16 if self.ctx.type == 'cuda' else torch.float32
        # bf16 (default), fp16 (BASELINE config 5's "fp16 MFMA path": v_mfma_f32_16x16x32_f16 in the
        # conv / FC kernels, fp16 activations through BN, pooling, RoIPool and the proposal decode,
        # fp32 accumulation and epilogue math) or fp32 (PyTorch ops; the reference runs fp32)
        if compute_dtype not in (torch.bfloat16, torch.float16, torch.float32):
            raise ValueError('compute_dtype must be torch.bfloat16, torch.float16 or torch.float32 (got %s)'
                             % compute_dtype)
        self.dtype = compute_dtype
        if self.ctx.type == 'cuda' and compute_dtype != torch.float32:
            self._to_lowp()

    def _to_lowp(self):
        from ..models.layers import Conv, Linear
        for m in self.model.modules():
            if isinstance(m, (Conv, Linear)):
                m.weight.data = m.weight.data.to(self.dtype)
                if m.weight.dim() == 4:
                    m.weight.data = m.weight.data.contiguous(memory_format=torch.channels_last)
                if m.bias is not None:
                    m.bias.data = m.bias.data.to(self.dtype)

    def _prep(self, im_array):
        x = torch.as_tensor(np.asarray(im_array) if not torch.is_tensor(im_array) else im_array)
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
        return self.model.detect(data, info, rois)

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
