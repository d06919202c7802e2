"""A whole training step as one HIP graph (``torch.cuda.graph`` over the step; the routing library records
its launches into the capture, ``capi.cpp: capturing``).

The C3 step -- parameter network, q' gather, routing forward, daily objective, routing backward, parameter
network backward, clip + Adam -- is ~40 launches and the Python between them; replaying it as one graph
removes the launch gaps and the host from the step (at a 112k-reach shard the gaps were ~0.15 ms of 6.2).

Requirements on ``fn`` (one training step): the same input tensors every step (copy new data into them in
place), an optimizer whose state lives on the device (:class:`ddr_amd.train.ClipAdam`, or
``torch.optim.Adam(capturable=True)``), no host synchronisation, no collective (all-reduce outside the graph),
no split-basin graph and no q' NaN check (the library refuses both under capture).  The routing graph must
have been used once before capture: the warm-up steps do that.
"""

from __future__ import annotations

import torch


class CapturedStep:
    """``fn`` run ``warmup`` times on a side stream, then captured; calling the object replays it."""

    def __init__(self, fn, warmup: int = 2, device: torch.device | None = None):
        dev = device or torch.device("cuda", torch.cuda.current_device())
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                fn()
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            fn()

    def __call__(self) -> None:
        self.graph.replay()
