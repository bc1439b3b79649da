"""Reference-compatible API facade (`rcnn.*` of walkoncross/mx-rcnn) over mx_rcnn_amd."""
