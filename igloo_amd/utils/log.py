"""Structured logging to stderr, level from ``IGLOO_LOG`` (debug|info|warn|error).

The reference has only println!/eprintln! and an unsubscribed ``tracing``
(SURVEY §5.1/5.5); this gives every component a named logger.
"""
from __future__ import annotations

import logging
import os
import sys

_CONFIGURED = False


def get_logger(name: str) -> logging.Logger:
    global _CONFIGURED
    if not _CONFIGURED:
        level = os.environ.get("IGLOO_LOG", "warning").upper()
        level = {"WARN": "WARNING"}.get(level, level)
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s igloo.%(name)s: %(message)s"))
        root = logging.getLogger("igloo")
        root.addHandler(h)
        root.setLevel(getattr(logging, level, logging.WARNING))
        root.propagate = False
        _CONFIGURED = True
    return logging.getLogger("igloo").getChild(name)
