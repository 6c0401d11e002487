"""hipGraph capture of whole training / inference steps (the MI355X answer to a
tracing compiler): a step that is launch-bound -- small graphs, dozens of
short kernels -- is captured once and replayed as one graph launch.

``StepGraph(fn)`` runs ``fn`` eagerly for ``warmup`` calls on a side stream
(so lazily allocated state -- optimizer moments, autograd buffers, hipBLASLt
workspaces -- exists before capture), then captures one call into a
``torch.cuda.CUDAGraph`` (a hipGraph on ROCm) and replays it for every later
call.  Everything the step reads must live in static tensors; the returned
tensors are the captured outputs, overwritten by each replay.  Randomness
inside the step must be graph-safe: PyTorch's Philox generator (dropout)
advances its offset per replay; the HIP kernels of this package read their
step counters from device memory.
"""
from __future__ import annotations

import gc
from typing import Any, Callable, Optional

import torch


class StepGraph:
    def __init__(self, fn: Callable[[], Any], warmup: int = 3, enabled: Optional[bool] = None,
                 device: Optional[torch.device] = None):
        self.fn = fn
        self.warmup = int(warmup)
        self.enabled = torch.cuda.is_available() if enabled is None else bool(enabled)
        self.device = device
        self.calls = 0
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.out: Any = None

    def _capture(self):
        # no garbage collection while capturing: a collected object that owns device
        # state (an older captured graph and its memory pool, an event) would make a
        # HIP call that is illegal inside a stream capture and abort the process
        gc.collect()
        was_enabled = gc.isenabled()
        gc.disable()
        try:
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.out = self.fn()
        finally:
            if was_enabled:
                gc.enable()

    def __call__(self):
        if not self.enabled:
            return self.fn()
        if self.graph is None:
            if self.calls < self.warmup:
                self.calls += 1
                s = torch.cuda.Stream(device=self.device)
                s.wait_stream(torch.cuda.current_stream(self.device))
                with torch.cuda.stream(s):
                    out = self.fn()
                torch.cuda.current_stream(self.device).wait_stream(s)
                return out
            self._capture()
        self.graph.replay()
        self.calls += 1
        return self.out

    def reset(self):
        """Drop the captured graph (e.g. after the step's shapes changed)."""
        self.graph, self.out, self.calls = None, None, 0
