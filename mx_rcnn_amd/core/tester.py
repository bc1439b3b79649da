"""Test loop (reference `rcnn/tester.py:10-136`): per image and class, score > 0.05 ->
NMS(TEST.NMS) -> at most 100 detections per image, scaled back to the original image; then
``imdb.evaluate_detections``.  Post-processing runs on the device (one batched per-class NMS
instead of C calls) and images can be batched.  Detections are cached as .npz."""
import logging
import os
import random

import numpy as np
import torch

from ..config import config
from ..processing import image_processing


def pred_eval(detector, test_data, imdb, vis=False, thresh=0.05, max_per_image=100, shard=(0, 1)):
    """``shard=(rank, world)``: ``test_data`` holds images ``rank::world`` of the image set (the
    reference tests on one GPU).  Per-rank detections are gathered and interleaved back into
    image order; rank 0 writes the cache and evaluates, and the result is broadcast so every
    rank returns the same value."""
    assert not test_data.shuffle
    rank, world = shard
    num_images = len(range(rank, imdb.num_images, world))
    all_boxes = [[np.zeros((0, 5), np.float32) for _ in range(num_images)] for _ in range(imdb.num_classes)]
    i = 0
    for batch in test_data:
        if i % 10 == 0:
            logging.info('testing %d/%d', i, num_images)
        if config.TEST.HAS_RPN:
            res = detector.detect_batch(batch['data'], batch['im_info'], thresh, config.TEST.NMS, max_per_image)
        else:
            res = detector.detect_batch(batch['data'], batch['im_info'], thresh, config.TEST.NMS, max_per_image,
                                        rois=batch['rois'])
        for boxes, scores, classes in res:
            if i >= num_images:
                break
            b, s, c = boxes.cpu().numpy(), scores.cpu().numpy(), classes.cpu().numpy()
            for j in range(1, imdb.num_classes):
                m = c == j
                all_boxes[j][i] = np.hstack((b[m], s[m, None])).astype(np.float32)
            if vis:
                dets = [[]] + [all_boxes[j][i] for j in range(1, imdb.num_classes)]
                vis_all_detection(batch['data'].numpy() if torch.is_tensor(batch['data']) else batch['data'],
                                  dets, imdb.classes)
            i += 1
    if world > 1:
        import torch.distributed as dist
        parts = [None] * world
        dist.all_gather_object(parts, all_boxes)
        num_images = imdb.num_images
        all_boxes = [[parts[k % world][j][k // world] for k in range(num_images)] for j in range(imdb.num_classes)]
        result = [None]
        if rank == 0:
            result[0] = _cache_and_evaluate(imdb, all_boxes)
        dist.broadcast_object_list(result, src=0)
        return result[0]
    return _cache_and_evaluate(imdb, all_boxes)


def _cache_and_evaluate(imdb, all_boxes):
    num_images = imdb.num_images
    if getattr(imdb, 'cache_path', None):
        cache_folder = os.path.join(imdb.cache_path, imdb.name)
        os.makedirs(cache_folder, exist_ok=True)
        np.savez(os.path.join(cache_folder, 'detections.npz'),
                 **{'c%d_i%d' % (j, k): all_boxes[j][k] for j in range(imdb.num_classes) for k in range(num_images)})
    return imdb.evaluate_detections(all_boxes)


def vis_all_detection(im_array, detections, imdb_classes=None, thresh=0.7):
    import matplotlib
    matplotlib.use('Agg')
    import matplotlib.pyplot as plt
    im = image_processing.transform_inverse(np.asarray(im_array)[:1], config.PIXEL_MEANS)
    plt.imshow(im)
    for j in range(1, len(imdb_classes)):
        color = (random.random(), random.random(), random.random())
        dets = detections[j]
        for k in range(len(dets)):
            bbox, score = dets[k, :4], dets[k, -1]
            if score > thresh:
                plt.gca().add_patch(plt.Rectangle((bbox[0], bbox[1]), bbox[2] - bbox[0], bbox[3] - bbox[1],
                                                  fill=False, edgecolor=color, linewidth=3.5))
                plt.gca().text(bbox[0], bbox[1] - 2, '{:s} {:.3f}'.format(imdb_classes[j], score),
                               bbox=dict(facecolor=color, alpha=0.5), fontsize=12, color='white')
    plt.savefig('vis.png')
    plt.close()


def draw_boxes(im_bgr, boxes, color=(0, 255, 0), width=2):
    """Rectangle drawing on a BGR uint8 image (replaces cv2.rectangle)."""
    im = im_bgr.copy()
    h, w = im.shape[:2]
    def cl(v, hi):
        return max(0, min(int(v), hi))
    for b in boxes:
        x1, y1, x2, y2 = [int(round(float(v))) for v in b[:4]]
        x1, x2, y1, y2 = cl(x1, w - 1), cl(x2, w - 1), cl(y1, h - 1), cl(y2, h - 1)
        for t in range(width):
            im[cl(y1 + t, h - 1), x1:x2 + 1] = color
            im[cl(y2 - t, h - 1), x1:x2 + 1] = color
            im[y1:y2 + 1, cl(x1 + t, w - 1)] = color
            im[y1:y2 + 1, cl(x2 - t, w - 1)] = color
    return im


def save_all_detection(im_array, detections, imdb_classes=None, thresh=0.7, path='result.jpg'):
    im = image_processing.transform_inverse(np.asarray(im_array)[:1], config.PIXEL_MEANS)
    im = im[:, :, ::-1].copy()
    for j in range(1, len(imdb_classes)):
        color = tuple(int(255 * random.random()) for _ in range(3))
        dets = detections[j]
        keep = [d for d in dets if d[-1] > thresh]
        im = draw_boxes(im, keep, color)
    image_processing.imwrite(path, im)
    return im
