"""RPN proposal generation / dump (reference `rcnn/rpn/generate.py:7-116`): runs the RPN test
graph and writes ``<root>/rpn_data/<imdb>_rpn.npz`` -- the hand-off from the RPN stage to the
R-CNN stage of alternate training (pickle-free, see data/cache.py)."""
import logging
import os

import numpy as np
import torch

from ..config import config
from ..data import cache as cache_io


class Detector(object):
    """RPN-only detector: ``im_detect(im, im_info) -> (boxes (n, 4) in input pixels, scores (n, 1))``."""

    def __init__(self, symbol, ctx=None, arg_params=None, aux_params=None, compute_dtype=None):
        from .detector import Detector as _D
        self._det = _D(symbol, ctx, arg_params, aux_params, compute_dtype)
        self.model = self._det.model

    @torch.no_grad()
    def im_detect(self, im, im_info):
        data = self._det._prep(im)
        info = torch.as_tensor(np.asarray(im_info) if not torch.is_tensor(im_info) else im_info).float()
        rois, scores = self._det.rpn_test(data, info.to(data.device))
        return rois[0, :, 1:].cpu().numpy(), scores[0, :, None].cpu().numpy()


def generate_detections(detector, test_data, imdb, vis=False, shard=(0, 1)):
    """Run the RPN over ``test_data`` and write the proposal dump.  ``shard=(rank, world)``:
    the iterator holds images ``rank::world`` of the image set; the per-rank lists are gathered
    (interleaved back into image order) and rank 0 writes the file."""
    assert not test_data.shuffle
    rank, world = shard
    imdb_boxes = []
    for i, batch in enumerate(test_data):
        if i % 10 == 0:
            logging.info('generating detections %d/%d', i * world + rank, imdb.num_images)
        boxes, scores = detector.im_detect(batch['data'], batch['im_info'])
        scale = float(batch['im_info'][0, 2])
        dets = np.hstack((boxes / scale, scores))
        imdb_boxes.append(dets)
        if vis:
            vis_detection(np.asarray(batch['data']), dets, thresh=0.9)
    if world > 1:
        import torch.distributed as dist
        parts = [None] * world
        dist.all_gather_object(parts, imdb_boxes)
        imdb_boxes = [parts[i % world][i // world] for i in range(sum(len(p) for p in parts))]
    assert len(imdb_boxes) == imdb.num_images, 'calculations not complete'
    rpn_folder = os.path.join(imdb.root_path, 'rpn_data')
    rpn_file = os.path.join(rpn_folder, imdb.name + '_rpn.npz')
    if rank == 0:
        os.makedirs(rpn_folder, exist_ok=True)
        cache_io.save_box_list(rpn_file, imdb_boxes)
        logging.info('wrote rpn proposals to %s', rpn_file)
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    return imdb_boxes


def vis_detection(im, dets, thresh=0.0):
    from .tester import save_all_detection
    save_all_detection(im, [[], dets[dets[:, -1] > thresh]], ['bg', 'obj'], thresh, path='rpn_vis.jpg')
