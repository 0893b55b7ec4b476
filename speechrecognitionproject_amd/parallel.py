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
    """Process-group settings for HIP-graph-captured collectives, set before any group exists.
    ProcessGroupNCCL recycles its work events through a per-device cache shared by all of its groups, so
    an event last recorded while a step was being captured could be handed to a later eager collective
    of another group, whose watchdog query would then fail on ROCm; TORCH_NCCL_CUDA_EVENT_CACHE=0 (an
    explicit setting is kept) gives every collective fresh events.  The cause of the round-4 watchdog
    abort was a different one (see ``capture_group``)."""
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")


def init_from_env(backend=None):
    """Initialise the default process group if WORLD_SIZE > 1; returns (rank, world, local_rank).
    Over RCCL the group is bound to this rank's GPU (``device_id``), which initialises its
    communicator eagerly and lets ``capture_group`` split a second one off it before any capture."""
    world, rank, local = env_world()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            nccl_env_for_graph_capture()
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        # a long timeout: rank 0 alone runs the reference's per-epoch accuracy passes while the other
        # ranks wait at a barrier (training.py)
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=int(os.environ.get("SRK_DIST_TIMEOUT", "7200"))),
                                **kw)
    elif torch.cuda.is_available():
        torch.cuda.set_device(local)
    return rank, world, local


_CAPTURE_GROUP = None


def capture_group():
    """The process group used ONLY by collectives recorded into HIP graphs (a collective call: every
    rank calls it, before any capture).

    Why a group of its own (the round-4 watchdog abort): ProcessGroupNCCL hands every
    EAGER collective's Work to its watchdog thread, which polls the Work's end event (recorded on the
    group's internal stream) until it sees it complete — on its own interval, so a Work can stay listed
    well after the device finished it.  A collective issued during a capture makes that same internal
    stream wait on the capturing stream, i.e. joins it to the capture, and on ROCm ``hipEventQuery`` of
    an event whose stream is now capturing fails with hipErrorCapturedEvent
    (tests/test_dp_graph_gpu.py::test_hip_rule_event_on_stream_joined_to_capture).  The watchdog
    rethrows that and aborts the process — whenever a capture started before it had reaped the warm-up
    steps' eager all-reduces.  A group that never runs an eager collective has no listed Work whose
    event could sit on its stream when a capture joins it (captured collectives are not handed to the
    watchdog), so the race cannot occur.  Over RCCL the group is split off the default group's
    communicator at creation (the default group is bound to a device, ``init_from_env``), so no
    communicator setup is left for the first captured collective either."""
    global _CAPTURE_GROUP
    if not (dist.is_available() and dist.is_initialized()):
        return None
    world_pg = dist.group.WORLD
    if _CAPTURE_GROUP is None or _CAPTURE_GROUP[0] is not world_pg:   # (re)initialised default group
        _CAPTURE_GROUP = (world_pg, dist.new_group(backend=dist.get_backend()))
    return _CAPTURE_GROUP[1]


def group_for_now(group=None):
    """The process group a collective issued at this point must run on: ``group`` eagerly, the
    capture-only group while the current stream is capturing a HIP graph (see ``capture_group``; it
    must already exist — creating a communicator under capture is not possible).  A capture of a
    collective on a non-default ``group`` has no capture-only counterpart and is refused."""
    if not (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()):
        return group
    if group is not None and group is not dist.group.WORLD:
        raise RuntimeError("a collective on a non-default process group cannot be captured safely "
                           "(DESIGN.md §4); run the step eagerly")
    if _CAPTURE_GROUP is None or _CAPTURE_GROUP[0] is not dist.group.WORLD:
        raise RuntimeError("a captured collective needs parallel.capture_group() created (on every rank) "
                           "before the capture starts (DESIGN.md §4)")
    return _CAPTURE_GROUP[1]


def world_size():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def barrier():
    if world_size() > 1:
        dist.barrier()


def broadcast_flat(flat):
    """Make every rank start from rank 0's parameters (one broadcast of the flat buffer)."""
    if world_size() > 1:
        dist.broadcast(flat.data, src=0)


def allreduce_grads(flat, at_world1=False):
    """Sum the flat gradient buffer over ranks (one collective per step).  The optimizer applies
    1/world through its grad_scale, so no separate scaling pass runs.  Inside a HIP-graph capture
    it runs on the capture-only group (``group_for_now``), never on the default group that the
    warm-up steps used eagerly.  ``at_world1`` issues it in a 1-rank group too (the GPU test of that
    capture on a one-GPU box)."""
    if world_size() > (0 if at_world1 else 1):
        dist.all_reduce(flat.grad, op=dist.ReduceOp.SUM, group=group_for_now())


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

    Streams: every collective is issued under the stream that was current when ``begin()`` ran (the
    compute stream of the step), also when ``_launch`` runs from a post-accumulate hook on autograd's
    device thread, whose current stream is whatever autograd chose for that node.

    HIP graphs: the whole step — forward, backward with these bucketed collectives, ``finish()`` and
    the optimizer — is captured into one graph (bench.py and training.py at N > 1 over RCCL).  The host
    logic above runs once, during the capture, so each collective is recorded at the point of the stream
    order where its bucket became final: a graph node on the process group's stream, forked from the
    compute stream there and joined back before the optimizer.  A step that ``begin()`` finds capturing
    issues its collectives on ``capture_group`` (pass ``parallel.capture_group()``, created eagerly on
    every rank), eager steps on ``group``: no collective of the capture group is ever run eagerly, which
    is what keeps the process group's watchdog away from events on a capturing stream (see
    ``capture_group``).  ``collectives_at_world1`` issues them even in a 1-rank group (the GPU test of
    that capture on a one-GPU box)."""

    def __init__(self, flat, bucket_mb=8.0, group=None, collectives_at_world1=False, capture_group=None):
        self.flat, self.group, self.capture_group = flat, group, capture_group
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
        """Reset per-step state; call before the forward pass of each step (on the step's stream)."""
        self.remaining = [len(ps) for _, _, ps in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.ready = set()
        self.works = []
        self.pending = 0
        self.held = []
        self.stream, self.capturing = None, False
        if self.flat.grad.is_cuda:
            self.stream = torch.cuda.current_stream(self.flat.grad.device)
            self.capturing = torch.cuda.is_current_stream_capturing()
        if self.capturing and self.capture_group is None and self._active(self.group):
            raise RuntimeError("GradReducer: a captured step needs capture_group=parallel.capture_group() "
                               "(an eager group's collectives cannot be captured safely, DESIGN.md §4)")

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

    def _active(self, group):
        return (dist.is_available() and dist.is_initialized()
                and dist.get_world_size(group) >= self.min_world)

    def _launch(self, i):
        if self.launched[i]:
            return
        self.launched[i] = True
        lo, hi, _ = self.buckets[i]
        group = self.capture_group if self.capturing else self.group
        if not self._active(group):
            return
        if self.stream is None:
            work = dist.all_reduce(self.flat.grad[lo:hi], op=dist.ReduceOp.SUM, group=group, async_op=True)
        else:
            with torch.cuda.stream(self.stream):
                work = dist.all_reduce(self.flat.grad[lo:hi], op=dist.ReduceOp.SUM, group=group, async_op=True)
        self.works.append(work)

    def finish(self):
        """Launch every bucket not launched yet (in bucket order) and wait for all of them."""
        self.pending = 0
        for i in range(len(self.buckets)):
            self._launch(i)
        if self.stream is None:
            for w in self.works:
                w.wait()
        else:
            with torch.cuda.stream(self.stream):
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
