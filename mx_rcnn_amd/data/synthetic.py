"""Synthetic image database: random images of a fixed shape with random boxes (the
"synthetic data of the named shape" used by the benchmarks and tests; no files needed).

Images are generated deterministically from a per-entry seed when loaded, so the roidb is
small and picklable-free."""
import numpy as np
import scipy.sparse

from .imdb import IMDB


class SyntheticDetection(IMDB):
    def __init__(self, num_images=16, height=600, width=1000, num_classes=21, max_gt=20, seed=0, name='synthetic'):
        super(SyntheticDetection, self).__init__(name)
        self.height, self.width = height, width
        self.num_classes = num_classes
        self.classes = ['__background__'] + ['class%d' % i for i in range(1, num_classes)]
        self.num_images = num_images
        self.image_set_index = list(range(num_images))
        self.max_gt = max_gt
        self.seed = seed

    def image_path_from_index(self, index):
        return None

    def image_size_from_index(self, index):
        return self.height, self.width

    def evaluate_detections(self, detections):
        from .voc_eval import eval_in_memory
        return eval_in_memory(self.gt_roidb(), detections, self.classes)

    def gt_roidb(self):
        rng = np.random.RandomState(self.seed)
        out = []
        for i in range(self.num_images):
            k = int(rng.randint(1, self.max_gt + 1))
            bw = rng.randint(16, max(17, self.width // 3), size=k)
            bh = rng.randint(16, max(17, self.height // 3), size=k)
            x1 = np.floor(rng.rand(k) * (self.width - bw - 1))
            y1 = np.floor(rng.rand(k) * (self.height - bh - 1))
            boxes = np.stack([x1, y1, x1 + bw, y1 + bh], 1).astype(np.uint16)
            cls = rng.randint(1, self.num_classes, size=k).astype(np.int32)
            ov = np.zeros((k, self.num_classes), np.float32)
            ov[np.arange(k), cls] = 1
            out.append({'boxes': boxes, 'gt_classes': cls, 'gt_overlaps': scipy.sparse.csr_matrix(ov),
                        'flipped': False, 'height': self.height, 'width': self.width,
                        'synthetic_seed': self.seed * 100003 + i})
        return out


def synthetic_image(entry):
    """BGR uint8 image for a synthetic roidb entry (textured noise + bright boxes)."""
    rng = np.random.RandomState(entry['synthetic_seed'] % (2 ** 31))
    h, w = entry['height'], entry['width']
    im = rng.randint(0, 255, size=(h, w, 3), dtype=np.uint8)
    boxes = np.asarray(entry['boxes'])
    cls = entry.get('gt_classes')
    if cls is not None:  # merged roidbs (alternate training) also hold proposal rows: draw the gt only
        boxes = boxes[np.asarray(cls) > 0]
    for b in boxes:
        x1, y1, x2, y2 = [int(v) for v in b]
        im[y1:y2 + 1, x1:x2 + 1] = (im[y1:y2 + 1, x1:x2 + 1] // 2 + 120).astype(np.uint8)
    return im
