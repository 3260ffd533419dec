"""`madpose.utils` compatibility alias (reference: madpose/utils.py)."""
from madpose_amd.utils import *  # noqa: F401,F403
