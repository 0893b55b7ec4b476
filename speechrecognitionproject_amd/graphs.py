"""HIP-graph replay of a warm-up-stable train step (training.py:83-95 minus its host work).

A train step of this package is a fixed sequence of launches on one stream (the HIP kernels behind
the C ABI, the persistent GRU's counter memsets, torch's allocator and autograd bookkeeping) whose
shapes, pointers and host arguments do not change from step to step once the batch shape is fixed:
the only per-step host values — the Adam step count and the dropout seed — live on the device
(``optim.Adam.state_dev``, ``nn._dropout_state``).  ``GraphedStep`` records that sequence once into a
HIP graph (torch.cuda.graph: a private memory pool, capture on a side stream) and then launches the
whole step with one ``hipGraphLaunch``, removing the per-kernel host launch cost.

Inputs must sit at fixed addresses: the caller copies each batch into ``static`` tensors it passes
to the step function, then calls ``replay()`` — or, when the batches are already resident (bench.py's
pre-staged pool), captures one graph per batch slot sharing one memory pool, which avoids the copy
(a device-to-device ``copy_`` goes through a DMA engine: measured +0.3-0.7 ms per 16 MB batch).

Constraints (checked by the parity tests, tests/test_graphs_gpu.py): every library scratch buffer must
already have its final size when the capture starts (the warm-up runs the step at least twice), and
the per-step kernel timers (srk_prof) stay off during capture and replay; bench.py times kernels in a
separate eager pass of the same step.
"""
import gc

import torch

from . import _lib


def _detached(out):
    """The step's output without its autograd graph: a replay only rewrites the tensor's memory, and a
    live graph would keep this capture's AccumulateGrad nodes (and their stream) into the next one."""
    if isinstance(out, torch.Tensor):
        return out.detach()
    if isinstance(out, (tuple, list)):
        return type(out)(_detached(o) for o in out)
    return out


class GraphedStep:
    """``step()`` -> its output tensor(s), captured after ``warmup`` eager calls on a side stream."""

    def __init__(self, step, warmup=2, pool=None, capture_error_mode="global"):
        """warmup: eager calls of ``step`` on a side stream before the capture (>= 2 so every scratch
        buffer reaches its size), or 0 when the caller has just run >= 2 steps of the same shapes on a
        side stream itself (training.py: real steps on real batches, no repeated step).
        capture_error_mode: torch.cuda.graph's; "thread_local" when the step issues RCCL collectives
        (the process group's watchdog thread keeps making runtime calls during the capture)."""
        if warmup == 1 or warmup < 0:
            raise ValueError("GraphedStep: warmup must be 0 (caller warmed up) or >= 2")
        self.step = step
        self.graph = None
        self.out = None
        if warmup:
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(warmup):
                    self.out = step()
            torch.cuda.current_stream().wait_stream(side)
        # drop the warm-up's output: its autograd graph would keep the side stream's AccumulateGrad
        # nodes alive into the capture (and collect any reference cycle still holding one)
        self.out = None
        gc.collect()
        torch.cuda.synchronize()
        self.generation = _lib.scratch_generation()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, pool=pool, capture_error_mode=capture_error_mode):
            out = step()
        self.out = _detached(out)
        del out
        torch.cuda.synchronize()
        if _lib.scratch_generation() != self.generation:
            raise _lib.SrkError("GraphedStep: a library scratch buffer grew during the capture (warm up longer)")

    def pool(self):
        """The graph's private memory pool: graphs captured with it share memory (replay them one at
        a time, as a training loop does)."""
        return self.graph.pool()

    def valid(self):
        """False once a library scratch buffer the graph may refer to has been reallocated."""
        return self.graph is not None and _lib.scratch_generation() == self.generation

    def replay(self):
        if not self.valid():
            raise _lib.SrkError("GraphedStep: the library's scratch buffers were reallocated after the capture "
                                "(another shape ran in between): capture again")
        self.graph.replay()
        return self.out

    def release(self):
        """Drop the graph and its private memory pool (before other shapes grow shared scratch)."""
        self.graph = None
        self.out = None
