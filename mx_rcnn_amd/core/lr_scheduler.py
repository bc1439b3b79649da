"""LR schedules counting optimizer updates (MXNet `num_update`).

* ``FactorScheduler(step, factor)``: base_lr * factor^(floor(n/step)) (mx.lr_scheduler).
* ``WarmupScheduler`` reproduces `rcnn/warmup.py:4-58`: constant warmup_lr for
  num_update < warmup_step, then base_lr, multiplied by factor every `step` updates.
"""
import logging


class LRScheduler(object):
    def __init__(self, base_lr=0.01):
        self.base_lr = base_lr

    def __call__(self, num_update):
        raise NotImplementedError


class FactorScheduler(LRScheduler):
    def __init__(self, step, factor=1.0, stop_factor_lr=1e-8):
        super().__init__()
        if step < 1:
            raise ValueError('Schedule step must be greater or equal than 1 round')
        if factor > 1.0:
            raise ValueError('Factor must be no more than 1 to make lr reduce')
        self.step, self.factor, self.stop_factor_lr = step, factor, stop_factor_lr
        self.count = 0

    def __call__(self, num_update):
        while num_update > self.count + self.step:
            self.count += self.step
            self.base_lr *= self.factor
            if self.base_lr < self.stop_factor_lr:
                self.base_lr = self.stop_factor_lr
            logging.info('Update[%d]: Change learning rate to %0.5e', num_update, self.base_lr)
        return self.base_lr


class WarmupScheduler(LRScheduler):
    def __init__(self, step, factor=1, warmup_lr=1e-5, warmup_step=500):
        super().__init__()
        if step < 1:
            raise ValueError('Schedule step must be greater or equal than 1 round')
        if factor > 1.0:
            raise ValueError('Factor must be no more than 1 to make lr reduce')
        self.step, self.factor = step, factor
        self.count = 0
        self.warmup_lr, self.warmup_step = warmup_lr, warmup_step
        self.normal_lr = None

    def __call__(self, num_update):
        if self.normal_lr is None:
            self.normal_lr = self.base_lr
        if num_update < self.warmup_step:
            return self.warmup_lr
        n = num_update - self.warmup_step
        lr = self.normal_lr * (self.factor ** (n // self.step)) if n > self.step else self.normal_lr
        if lr != self.base_lr:
            logging.info('Update[%d]: Change learning rate to %0.5e', num_update, lr)
        self.base_lr = lr
        return lr
