"""Training metrics (reference `rcnn/metric.py:12-126`) accumulated ON THE DEVICE.

The reference calls ``.asnumpy()`` on every output every batch (6 host syncs per step);
here ``update`` only launches small reductions into device accumulators and ``get()``
(called every ``frequent`` batches by the Speedometer) is the only host read.
Names and definitions match: RPN-Accuracy / RPN-LogLoss / RPN-SmoothL1Loss (per image) and
Accuracy / LogLoss / SmoothL1Loss (per RoI) of approximate-joint training.
"""
import torch

from ..config import config


class EvalMetric(object):
    def __init__(self, name):
        self.name = name
        self.reset()

    def reset(self):
        self.sum_metric = None
        self.num_inst = None

    def _acc(self, s, n):
        s = s.detach().double().reshape(())
        n = torch.as_tensor(n, dtype=torch.float64, device=s.device).reshape(())
        if self.sum_metric is None:
            self.sum_metric, self.num_inst = s.clone(), n.clone()
        else:
            self.sum_metric += s
            self.num_inst += n

    def get(self):
        if self.sum_metric is None:
            return self.name, float('nan')
        n = float(self.num_inst)
        return self.name, (float(self.sum_metric) / n) if n > 0 else float('nan')

    def get_name_value(self):
        name, value = self.get()
        return [(name, value)]


def _rpn_view(out):
    score = out['rpn_cls_score']
    B, C2, H, W = score.shape
    return score.float().reshape(B, 2, (C2 // 2) * H, W), out['rpn_label'].reshape(B, (C2 // 2) * H, W)


class AccuracyMetric(EvalMetric):
    def __init__(self, use_ignore=False, ignore=None, ex_rpn=False):
        self.use_ignore, self.ignore, self.ex_rpn = use_ignore, ignore, ex_rpn
        super().__init__('RPN-Accuracy' if ex_rpn else 'Accuracy')

    def update(self, labels, preds):
        out = preds
        with torch.no_grad():
            if self.ex_rpn:
                if 'rpn_cls_score' not in out:
                    return
                score, label = _rpn_view(out)
                pred = score.argmax(dim=1)
                valid = label != (self.ignore if self.ignore is not None else -1)
                self._acc(((pred == label) & valid).sum(), valid.sum())
            else:
                if 'cls_prob' not in out:
                    return
                pred = out['cls_prob'].argmax(dim=1)
                label = out['label'].long()
                self._acc((pred == label).sum(), label.numel())


class LogLossMetric(EvalMetric):
    def __init__(self, use_ignore=False, ignore=None, ex_rpn=False):
        self.use_ignore, self.ignore, self.ex_rpn = use_ignore, ignore, ex_rpn
        super().__init__('RPN-LogLoss' if ex_rpn else 'LogLoss')

    def update(self, labels, preds):
        out = preds
        with torch.no_grad():
            if self.ex_rpn:
                if 'rpn_cls_score' not in out:
                    return
                score, label = _rpn_view(out)
                prob = torch.softmax(score, dim=1)
                valid = label != (self.ignore if self.ignore is not None else -1)
                p = prob.gather(1, label.clamp_min(0).long()[:, None])[:, 0]
                self._acc((-torch.log(p + config.EPS) * valid).sum(), valid.sum())
            else:
                if 'cls_prob' not in out:
                    return
                label = out['label'].long()
                p = out['cls_prob'].gather(1, label.clamp_min(0)[:, None])[:, 0]
                self._acc((-torch.log(p + config.EPS)).sum(), label.numel())


class SmoothL1LossMetric(EvalMetric):
    def __init__(self, ex_rpn=False):
        self.ex_rpn = ex_rpn
        super().__init__('RPN-SmoothL1Loss' if ex_rpn else 'SmoothL1Loss')

    def update(self, labels, preds):
        out = preds
        if self.ex_rpn:
            if 'rpn_bbox_loss' in out:
                self._acc(out['rpn_bbox_loss'], out['num_images'])
        elif 'bbox_loss' in out:
            self._acc(out['bbox_loss'], out['num_rois'])


class CompositeEvalMetric(EvalMetric):
    def __init__(self, metrics=None):
        self.metrics = list(metrics or [])
        super().__init__('composite')

    def add(self, metric):
        self.metrics.append(metric)

    def reset(self):
        for m in getattr(self, 'metrics', []):
            m.reset()

    def update(self, labels, preds):
        for m in self.metrics:
            m.update(labels, preds)

    def get(self):
        names, values = [], []
        for m in self.metrics:
            n, v = m.get()
            names.append(n)
            values.append(v)
        return names, values

    def get_name_value(self):
        n, v = self.get()
        return list(zip(n, v))


def e2e_metrics():
    """The six metrics of end-to-end training (train_end2end.py / train_widerface.py `metric()`)."""
    return CompositeEvalMetric([AccuracyMetric(use_ignore=True, ignore=-1, ex_rpn=True),
                                LogLossMetric(use_ignore=True, ignore=-1, ex_rpn=True),
                                SmoothL1LossMetric(ex_rpn=True), AccuracyMetric(), LogLossMetric(),
                                SmoothL1LossMetric()])


def rpn_metrics():
    return CompositeEvalMetric([AccuracyMetric(use_ignore=True, ignore=-1, ex_rpn=True),
                                LogLossMetric(use_ignore=True, ignore=-1, ex_rpn=True),
                                SmoothL1LossMetric(ex_rpn=True)])


def rcnn_metrics():
    return CompositeEvalMetric([AccuracyMetric(), LogLossMetric(), SmoothL1LossMetric()])
