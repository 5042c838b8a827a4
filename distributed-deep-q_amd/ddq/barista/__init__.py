"""Barista worker package: the reference's ``barista`` (barista/__init__.py,
constants.py) on the MI355X path.  Same constants, same module layout."""
import numpy as np

STATE_MD_LAYER = 0          # barista/constants.py:4-6 (memory-data layer indices)
NEXT_STATE_MD_LAYER = 1
ACTION_REWARD_MD_LAYER = 2

NUM_ACTIONS = 4             # constants.py:8
DTYPE = np.float32          # constants.py:9
DTYPE_SIZE = 4              # constants.py:10

MSG_LENGTH = 1              # constants.py:12
GRAD_UPDATE = b"G"          # constants.py:13 (one request byte on the wire)
DARWIN_UPDATE = b"D"        # constants.py:14
