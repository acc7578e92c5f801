"""MI355X-native per-frame Mask R-CNN hot path."""
import os

# MIOpen's Find evaluates every applicable convolution solver (NORMAL) instead of
# the default hybrid mode's dynamic subset: the body convs pick faster kernels
# (221 -> 225 frames/s measured on the default bench, profiles/r02c/).  A
# caller's own setting wins.  Read by MIOpen at its first Find, i.e. after this.
os.environ.setdefault("MIOPEN_FIND_MODE", "1")

# MIOpen's Find results for every benched configuration (R-50/R-101/X-101-FPN, C4,
# VOS; 155 convolution problems) recorded once on an MI355X (gfx950, 256 CUs) and
# shipped in-tree: every process -- each rank of a multi-GPU run, every box -- then
# picks the same solvers (identical numerics and per-rank speed) and skips the
# Find sweep at warm-up.  Problems not in it are found and appended as usual.  A
# caller's own MIOPEN_USER_DB_PATH wins.
os.environ.setdefault("MIOPEN_USER_DB_PATH",
                      os.path.join(os.path.dirname(os.path.abspath(__file__)), "miopen_db"))

