"""MI355X-native per-frame Mask R-CNN hot path."""
import os

# MIOpen's Find evaluates every applicable convolution solver (NORMAL) instead of
# the default hybrid mode's dynamic subset: the body convs pick faster kernels
# (221 -> 225 frames/s measured on the default bench, profiles/r02c/).  A
# caller's own setting wins.  Read by MIOpen at its first Find, i.e. after this.
os.environ.setdefault("MIOPEN_FIND_MODE", "1")
