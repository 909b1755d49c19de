"""Experiment transform (tools/exp_build.sh): gcn_fused.hip as committed at HEAD (for a same-box A/B
of the working tree's changes); reads the HEAD copy written to /tmp/ft/head_gcn_fused.hip."""
import shutil
import sys

shutil.copy("/tmp/ft/head_gcn_fused.hip", sys.argv[1])
