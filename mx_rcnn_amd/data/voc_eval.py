"""PASCAL VOC AP (reference `helper/dataset/voc_eval.py:10-178`) without the reference's two
live ``pdb.set_trace()`` traps and with the non-07 ``voc_ap`` concatenate bug fixed
(SURVEY §7.4 item 8).  Annotation cache is JSON (no pickle)."""
import json
import logging
import os
import xml.etree.ElementTree as ET

import numpy as np


def parse_voc_rec(filename):
    tree = ET.parse(filename)
    objects = []
    for obj in tree.findall('object'):
        bbox = obj.find('bndbox')
        diff = obj.find('difficult')
        objects.append({'name': obj.find('name').text,
                        'difficult': int(diff.text) if diff is not None else 0,
                        'bbox': [int(float(bbox.find(t).text)) for t in ('xmin', 'ymin', 'xmax', 'ymax')]})
    return objects


def voc_ap(rec, prec, use_07_metric=False):
    rec = np.asarray(rec, dtype=np.float64)
    prec = np.asarray(prec, dtype=np.float64)
    if use_07_metric:
        ap = 0.0
        for t in np.arange(0.0, 1.1, 0.1):
            p = 0.0 if np.sum(rec >= t) == 0 else np.max(prec[rec >= t])
            ap += p / 11.0
        return ap
    mrec = np.concatenate(([0.0], rec, [1.0]))
    mpre = np.concatenate(([0.0], prec, [0.0]))
    for i in range(mpre.size - 1, 0, -1):
        mpre[i - 1] = max(mpre[i - 1], mpre[i])
    i = np.where(mrec[1:] != mrec[:-1])[0]
    return float(np.sum((mrec[i + 1] - mrec[i]) * mpre[i + 1]))


def voc_eval(detpath, annopath, imageset_file, classname, cache_dir, ovthresh=0.5, use_07_metric=False):
    """-> (rec, prec, ap) for one class from a ``<id> score x1 y1 x2 y2`` results file."""
    os.makedirs(cache_dir, exist_ok=True)
    cache_file = os.path.join(cache_dir, 'annotations.json')
    with open(imageset_file) as f:
        image_filenames = [x.strip() for x in f.readlines() if x.strip()]
    recs = None
    if os.path.isfile(cache_file):
        with open(cache_file) as f:
            recs = json.load(f)
        if not all(k in recs for k in image_filenames):
            recs = None
    if recs is None:
        recs = {}
        for ind, name in enumerate(image_filenames):
            recs[name] = parse_voc_rec(annopath.format(name))
            if ind % 100 == 0:
                logging.info('reading annotations for %d/%d', ind + 1, len(image_filenames))
        with open(cache_file, 'w') as f:
            json.dump(recs, f)
    class_recs = {}
    npos = 0
    for name in image_filenames:
        objects = [o for o in recs[name] if o['name'] == classname]
        bbox = np.array([o['bbox'] for o in objects]).reshape(-1, 4)
        difficult = np.array([o['difficult'] for o in objects]).astype(bool)
        npos += int(np.sum(~difficult))
        class_recs[name] = {'bbox': bbox, 'difficult': difficult, 'det': [False] * len(objects)}
    with open(detpath.format(classname)) as f:
        split = [x.strip().split(' ') for x in f.readlines() if x.strip()]
    image_ids = [x[0] for x in split]
    confidence = np.array([float(x[1]) for x in split])
    bbox = np.array([[float(z) for z in x[2:]] for x in split]).reshape(-1, 4)
    return match_detections(class_recs, image_ids, confidence, bbox, npos, ovthresh, use_07_metric)


def match_detections(class_recs, image_ids, confidence, bbox, npos, ovthresh=0.5, use_07_metric=False):
    """Greedy score-ordered matching of detections to (non-difficult) gt -> (rec, prec, ap).
    ``class_recs[id] = {'bbox': (n,4), 'difficult': (n,) bool, 'det': [False]*n}``."""
    order = np.argsort(-confidence, kind='stable')
    bbox = bbox[order, :]
    image_ids = [image_ids[x] for x in order]
    nd = len(image_ids)
    tp = np.zeros(nd)
    fp = np.zeros(nd)
    for d in range(nd):
        r = class_recs[image_ids[d]]
        bb = bbox[d, :].astype(float)
        ovmax = -np.inf
        bbgt = r['bbox'].astype(float)
        jmax = -1
        if bbgt.size > 0:
            ixmin = np.maximum(bbgt[:, 0], bb[0])
            iymin = np.maximum(bbgt[:, 1], bb[1])
            ixmax = np.minimum(bbgt[:, 2], bb[2])
            iymax = np.minimum(bbgt[:, 3], bb[3])
            iw = np.maximum(ixmax - ixmin + 1., 0.)
            ih = np.maximum(iymax - iymin + 1., 0.)
            inters = iw * ih
            uni = ((bb[2] - bb[0] + 1.) * (bb[3] - bb[1] + 1.) +
                   (bbgt[:, 2] - bbgt[:, 0] + 1.) * (bbgt[:, 3] - bbgt[:, 1] + 1.) - inters)
            overlaps = inters / uni
            ovmax = np.max(overlaps)
            jmax = int(np.argmax(overlaps))
        if ovmax > ovthresh:
            if not r['difficult'][jmax]:
                if not r['det'][jmax]:
                    tp[d] = 1.
                    r['det'][jmax] = True
                else:
                    fp[d] = 1.
        else:
            fp[d] = 1.
    fp = np.cumsum(fp)
    tp = np.cumsum(tp)
    rec = tp / float(max(npos, 1))
    prec = tp / np.maximum(tp + fp, np.finfo(np.float64).eps)
    return rec, prec, voc_ap(rec, prec, use_07_metric)


def eval_in_memory(gt_roidb, detections, classes, ovthresh=0.5, use_07_metric=False):
    """mAP of ``detections[cls][img] = (n, 5)`` against in-memory gt entries (boxes, gt_classes)
    -- the evaluator for datasets without VOC annotation files (synthetic, .lst lists)."""
    aps = []
    for c in range(1, len(classes)):
        class_recs, npos = {}, 0
        for i, r in enumerate(gt_roidb):
            m = np.asarray(r['gt_classes']) == c
            bb = np.asarray(r['boxes'])[m].astype(float).reshape(-1, 4)
            class_recs[i] = {'bbox': bb, 'difficult': np.zeros(len(bb), bool), 'det': [False] * len(bb)}
            npos += len(bb)
        ids, conf, boxes = [], [], []
        for i in range(len(gt_roidb)):
            d = detections[c][i] if len(detections[c]) > i else []
            d = np.asarray(d, dtype=np.float64).reshape(-1, 5)
            ids += [i] * len(d)
            conf.append(d[:, 4])
            boxes.append(d[:, :4])
        conf = np.concatenate(conf) if conf else np.zeros(0)
        boxes = np.concatenate(boxes) if boxes else np.zeros((0, 4))
        _, _, ap = match_detections(class_recs, ids, conf, boxes, npos, ovthresh, use_07_metric)
        if npos > 0:
            aps.append(ap)
        logging.info('AP for %s = %.4f', classes[c], ap)
    mean_ap = float(np.mean(aps)) if aps else 0.0
    logging.info('Mean AP = %.4f', mean_ap)
    return mean_ap
