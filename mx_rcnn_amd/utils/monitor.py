"""Norm monitor (reference ``--monitor``: ``mx.mon.Monitor(100, norm_stat)`` installed through
``MutableModule.install_monitor``, `train_end2end.py:111-114`, `rcnn/module.py:197-200`).

Every ``interval`` steps it reports ``norm(x)/sqrt(x.size)`` of every named layer output,
weight and weight gradient.  Stats are reduced ON THE DEVICE during the step and read back
with one synchronisation in ``toc`` (the reference's per-array ``asnumpy``).  Forward hooks do
not run inside a replayed hipGraph, so ``MutableModule`` runs monitored steps eagerly and all
other steps from the graph.
"""
import logging
import re

import torch


def norm_stat(x):
    x = x.detach().float()
    return x.norm() / (x.numel() ** 0.5)


class Monitor(object):
    def __init__(self, interval=100, stat_func=None, pattern='.*', sort=False):
        self.interval = int(interval)
        self.stat_func = stat_func or norm_stat
        self.re = re.compile(pattern)
        self.sort = sort
        self.step = 0
        self.activated = False
        self.queue = []
        self.model = None
        self._handles = []

    def install(self, model):
        self.model = model
        for m in model.modules():
            name = getattr(m, 'mx_name', None)
            if name is None or not hasattr(m, 'mx_args'):
                continue
            self._handles.append(m.register_forward_hook(self._hook(name + '_output')))

    def _hook(self, name):
        def fn(mod, inp, out):
            if self.activated and self.re.match(name):
                t = out[0] if isinstance(out, (tuple, list)) else out
                if torch.is_tensor(t):
                    self.queue.append((self.step, name, self.stat_func(t)))
        return fn

    def is_active_next(self):
        return self.step % self.interval == 0

    def tic(self):
        if self.step % self.interval == 0:
            self.queue = []
            self.activated = True
        self.step += 1

    def toc(self):
        if not self.activated:
            return []
        if self.model is not None:
            for m in self.model.modules():
                name = getattr(m, 'mx_name', None)
                if name is None or not hasattr(m, 'mx_args'):
                    continue
                for attr, p in m._parameters.items():
                    if p is None:
                        continue
                    n = '%s_%s' % (name, attr)
                    if self.re.match(n):
                        self.queue.append((self.step, n, self.stat_func(p)))
                    if p.grad is not None and self.re.match(n + '_grad'):
                        self.queue.append((self.step, n + '_grad', self.stat_func(p.grad)))
        self.activated = False
        stats = torch.stack([v for _, _, v in self.queue]).cpu().tolist() if self.queue else []  # one sync
        res = [(s, n, '%.8f' % v) for (s, n, _), v in zip(self.queue, stats)]
        if self.sort:
            res.sort(key=lambda r: r[1])
        self.queue = []
        return res

    def toc_print(self):
        for s, n, v in self.toc():
            logging.info('Batch: %7d %30s %s', s, n, v)

    def remove(self):
        for h in self._handles:
            h.remove()
        self._handles = []
