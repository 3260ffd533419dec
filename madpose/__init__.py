"""`import madpose` compatibility alias for madpose_amd (reference: madpose/__init__.py:1)."""
from madpose_amd import *  # noqa: F401,F403
from madpose_amd import utils  # noqa: F401
