"""Datasets (PASCAL VOC, .lst detection lists, synthetic), roidb preparation, minibatch
construction and prefetching loaders (reference L2/L3: `helper/dataset/*`,
`helper/processing/roidb.py`, `utils/load_data.py`, `rcnn/minibatch.py`, `rcnn/loader.py`)."""
