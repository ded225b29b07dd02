"""glog-style logging with `-v` verbosity (reference logs device-plugin traffic at V(2)-V(5),
e.g. pkg/kubelet/cm/devicemanager/manager.go:128,138,141)."""
from __future__ import annotations

import logging
import sys

VERBOSITY = 0


def setup(v: int = 0, component: str = "amdkube"):
    global VERBOSITY
    VERBOSITY = v
    logging.basicConfig(stream=sys.stderr, level=logging.DEBUG if v >= 4 else logging.INFO,
                        format=f"%(levelname).1s%(asctime)s.%(msecs)03d {component} %(name)s] %(message)s",
                        datefmt="%m%d %H:%M:%S")


def V(level: int) -> bool:
    return VERBOSITY >= level
