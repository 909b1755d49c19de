"""Drop-in for the reference's ``model.py``: put this directory on ``sys.path`` ahead of the
reference tree and ``from model import *`` / ``gwnet(...)`` resolve to the libgwn implementation."""
from gwn_amd.model import gcn, gcn2, gwnet, gwnet_diff_G, linear, nconv, nconv2  # noqa: F401
