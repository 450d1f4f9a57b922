"""decorator.py:14-37 equivalents: ``NoSyncBase.no_sync`` and ``main_rank_only``."""

from __future__ import annotations

import contextlib


class NoSyncBase:
    def no_sync(self):
        """Skip the gradient all-reduce for this micro-batch (gradient accumulation).

        With the native data-parallel wrapper (pizero_native.ddp.PiZeroDDP) the
        wrapper's own no_sync is used; on a bare model this is a no-op context.
        """
        wrapper = getattr(self, "_ddp_wrapper", None)
        if self.use_ddp and wrapper is not None:
            return wrapper.no_sync()
        return contextlib.nullcontext()


def main_rank_only(func):
    def wrapper(*args, **kwargs):
        if not kwargs.get("main_rank", False):
            return None
        return func(*args, **kwargs)

    return wrapper
