from mx_rcnn_amd.data.imdb import IMDB  # noqa: F401
