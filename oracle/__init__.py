"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/oracle.py).  Never imported by spectralmc_amd."""
from .oracle import *  # noqa: F401,F403
from .oracle import build, lib  # noqa: F401
