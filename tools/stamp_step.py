#!/usr/bin/env python3
"""tools/stamp_probe.py step (one cfg3 train step, every instrumented launch stamped)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import stamp_probe  # noqa: E402

stamp_probe.step()
