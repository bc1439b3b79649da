#!/bin/bash
# Evaluate the end-to-end model (reference test.sh; --end2end is accepted here).
python test.py --has_rpn --end2end --prefix model/e2e --epoch 10 "$@"
