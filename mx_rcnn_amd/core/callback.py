"""Speedometer (reference `rcnn/callback.py:6-36`): logs ``samples/sec`` = global images/s
every ``frequent`` batches with the metric values, in the reference's log-line format, and
optionally appends a JSON line (imgs/s, per-stage ms) for the bench harness."""
import json
import logging
import time

from ..utils import profiler as prof


class BatchEndParam(object):
    def __init__(self, epoch, nbatch, eval_metric, locals=None):
        self.epoch, self.nbatch, self.eval_metric, self.locals = epoch, nbatch, eval_metric, locals


class Speedometer(object):
    def __init__(self, batch_size, frequent=50, jsonl=None):
        self.batch_size = batch_size
        self.frequent = frequent
        self.init = False
        self.tic = 0
        self.last_count = 0
        self.jsonl = jsonl
        self.last_speed = None

    def __call__(self, param):
        count = param.nbatch
        if self.last_count > count:
            self.init = False
        self.last_count = count
        if self.init:
            if count % self.frequent == 0:
                speed = self.frequent * self.batch_size / (time.time() - self.tic)
                self.last_speed = speed
                if param.eval_metric is not None:
                    names, values = param.eval_metric.get()
                    msg = '\t'.join('Train-%s=%f' % (n, v) for n, v in zip(names, values))
                    logging.info('Epoch[%d] Batch [%d]\tSpeed: %.2f samples/sec\t%s', param.epoch, count, speed, msg)
                else:
                    names, values = [], []
                    logging.info('Iter[%d] Batch [%d]\tSpeed: %.2f samples/sec', param.epoch, count, speed)
                stages = prof.report() if prof.enabled() else None
                if stages:
                    logging.info('Epoch[%d] Batch [%d]\tStages: %s', param.epoch, count, prof.format_report(stages))
                if self.jsonl:
                    with open(self.jsonl, 'a') as f:
                        f.write(json.dumps({'epoch': param.epoch, 'batch': count, 'samples_per_sec': speed,
                                            'metrics': dict(zip(names, values)),
                                            'stage_ms': stages or {}}) + '\n')
                self.tic = time.time()
        else:
            self.init = True
            self.tic = time.time()
