"""Data parallelism for the train step: one process per GPU, the per-clip batch
sharded across ranks, ONE all-reduce(SUM) of the flat fp32 gradient buffer per step through
RCCL (torch.distributed backend "nccl" on ROCm = RCCL over xGMI), 1/world folded into Adam.

The reference has no distributed code; this is new work required by
north_star.  Ranks are launched by ``torch.distributed.run`` (RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT in the environment).  On a CPU-only host the same code runs over gloo
(tests/test_parallel.py).
"""
import datetime
import os

import torch
import torch.distributed as dist


def env_world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def nccl_env_for_graph_capture():
    """Process-group settings for the (opt-in) HIP-graph-captured collectives, set before the group
    exists.  ProcessGroupNCCL recycles its work events through a cache, so an event last recorded while a
    step was being captured could be handed to a later eager collective, whose watchdog query would fail
    on ROCm ("operation not permitted on an event last recorded in a capturing stream") and abort the
    process.  TORCH_NCCL_CUDA_EVENT_CACHE=0 (an explicit setting is kept) gives every collective fresh
    events; the abort still recurred in the 1-rank capture test, which is why the captured form is opt-in
    (DESIGN.md §4)."""
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")


def init_from_env(backend=None):
    """Initialise the default process group if WORLD_SIZE > 1; returns (rank, world, local_rank)."""
    world, rank, local = env_world()
    nccl_env_for_graph_capture()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        # a long timeout: rank 0 alone runs the reference's per-epoch accuracy passes while the other
        # ranks wait at a barrier (training.py)
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=int(os.environ.get("SRK_DIST_TIMEOUT", "7200"))))
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return rank, world, local


def world_size():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def barrier():
    if world_size() > 1:
        dist.barrier()


def broadcast_flat(flat):
    """Make every rank start from rank 0's parameters (one broadcast of the flat buffer)."""
    if world_size() > 1:
        dist.broadcast(flat.data, src=0)


def allreduce_grads(flat):
    """Sum the flat gradient buffer over ranks (one collective per step).  The optimizer applies
    1/world through its grad_scale, so no separate scaling pass runs."""
    if world_size() > 1:
        dist.all_reduce(flat.grad, op=dist.ReduceOp.SUM)


class GradReducer:
    """Bucketed all-reduce of a FlatParams gradient buffer, overlapped with the backward pass
    (SURVEY.md §8e "overlap it with the backward pass").

    The flat buffer is cut into contiguous buckets of ~bucket_mb, built from the END of the
    parameter list (backward produces the last layers' gradients first).  A bucket's
    ``all_reduce(SUM, async_op=True)`` is launched as soon as every parameter in it has its
    gradient: autograd's post-accumulate hook for layers that return gradients, ``mark_ready`` from
    the GRU / Linear backward that accumulate into the buffer in place (nn.py).  The collective runs
    on the process group's own stream, which first waits for the compute stream, so it overlaps the
    backward work enqueued after it.

    Persistent kernels need every workgroup co-resident (csrc/gru_persistent.hip): a collective
    kernel sharing the CUs with one could starve it.  Each GRU layer forward calls
    ``persistent_pending(+1)``; its backward calls ``persistent_done`` right after enqueueing the
    recurrence: until the last such backward is enqueued, ready buckets are held (a collective
    launched afterwards waits for that kernel on the compute stream).  ``finish()`` launches what
    is left in bucket order (identical on every rank) and makes the compute stream wait for all.

    HIP graphs: the whole step — forward, backward with these bucketed collectives, ``finish()`` and
    the optimizer — can be captured into one graph (bench.py at N > 1).  The host logic above runs once,
    during the capture, so each collective is recorded at the point of the stream order where its bucket
    became final: a graph node on the process group's stream, forked from the compute stream there and
    joined back before the optimizer.  ``collectives_at_world1`` issues them even in a 1-rank group
    (the GPU test of that capture on a one-GPU box)."""

    def __init__(self, flat, bucket_mb=8.0, group=None, collectives_at_world1=False):
        self.flat, self.group = flat, group
        self.min_world = 1 if collectives_at_world1 else 2
        cap = max(1, int(bucket_mb * (1 << 20) / 4))
        groups, cur, size = [], [], 0
        for off, p in sorted(zip(flat.offsets, flat.params), key=lambda t: t[0], reverse=True):
            cur.append((off, p))
            size += p.numel()
            if size >= cap:
                groups.append(cur)
                cur, size = [], 0
        if cur:
            groups.append(cur)
        # contiguous cover of the buffer (alignment padding included): the first bucket ends at numel,
        # each later one where the previous one starts, the last one starts at 0
        self.buckets, end = [], flat.numel
        for gi, g in enumerate(groups):
            start = 0 if gi == len(groups) - 1 else min(off for off, _ in g)
            self.buckets.append((start, end, [p for _, p in g]))
            end = start
        self.bucket_of = {}
        for i, (_, _, ps) in enumerate(self.buckets):
            for p in ps:
                self.bucket_of[id(p)] = i
        self.hooks = [p.register_post_accumulate_grad_hook(self._hook) for p in flat.params]
        flat.reducer = self
        self.begin()

    def begin(self):
        """Reset per-step state; call before the forward pass of each step."""
        self.remaining = [len(ps) for _, _, ps in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.ready = set()
        self.works = []
        self.pending = 0
        self.held = []

    def persistent_pending(self, n=1):
        self.pending += n

    def persistent_done(self):
        self.pending = max(0, self.pending - 1)
        if self.pending == 0:
            held, self.held = self.held, []
            for i in held:
                self._launch(i)

    def _hook(self, p):
        self.mark_ready([p])

    def mark_ready(self, params):
        # idempotent per step: a layer that accumulates into .grad in place calls mark_ready after
        # enqueueing its GEMMs, and autograd STILL runs that parameter's post-accumulate hook (with no
        # gradient to add) afterwards; counting both would declare a bucket complete while some of
        # its gradients are still to be computed and launch its all-reduce too early
        for p in params:
            i = self.bucket_of.get(id(p))
            if i is None or id(p) in self.ready:
                continue
            self.ready.add(id(p))
            self.remaining[i] -= 1
            if self.remaining[i] == 0:
                if self.pending > 0:
                    self.held.append(i)
                else:
                    self._launch(i)

    def _launch(self, i):
        if self.launched[i]:
            return
        self.launched[i] = True
        lo, hi, _ = self.buckets[i]
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) >= self.min_world:
            self.works.append(dist.all_reduce(self.flat.grad[lo:hi], op=dist.ReduceOp.SUM, group=self.group,
                                              async_op=True))

    def finish(self):
        """Launch every bucket not launched yet (in bucket order) and wait for all of them."""
        self.pending = 0
        for i in range(len(self.buckets)):
            self._launch(i)
        for w in self.works:
            w.wait()
        self.works = []

    def remove(self):
        for h in self.hooks:
            h.remove()
        self.flat.reducer = None


def shard_indices(n_items, rank, world, seed, epoch=0):
    """DistributedSampler-equivalent: a seeded permutation, rank r takes every world-th item
    starting at r (padded by wrap-around so every rank gets the same count)."""
    g = torch.Generator().manual_seed(seed + epoch)
    perm = torch.randperm(n_items, generator=g)
    per = (n_items + world - 1) // world
    total = per * world
    if total > n_items:
        perm = torch.cat([perm, perm[: total - n_items]])
    return perm[rank:total:world]
