"""Worker of tests/test_dp_graph_gpu.py (run as a subprocess: it owns a 1-rank RCCL process group).

bench.py and training.py at N > 1 capture the whole DP step into a HIP graph: forward, backward with
the bucketed all-reduces of parallel.GradReducer forked where each bucket's gradients are final (on the
capture-only process group, parallel.capture_group), the join, and Adam.  On a one-GPU box the closest check is a 1-rank "nccl" (RCCL) group with the reducer
told to issue its collectives anyway: the captured step must then replay the eager step bit for bit
(a 1-rank SUM is the identity), buckets must be forked during the backward (not all at finish()),
and a captured collective must actually run on replay (a 1-rank all-gather copies a fresh input).
Mode "flat_syncbn" (ADVICE r05): no reducer — the single flat all-reduce of ``--no-overlap`` — and
SyncBatchNorm1d's statistics / backward sums, all captured right after eager warm-up steps on the
default group; parallel.group_for_now must put the captured ones on the capture-only group.
Prints one JSON line."""
import json
import os
import socket
import sys

import torch
import torch.distributed as dist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def main():
    name, B, precision = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    mode = sys.argv[4] if len(sys.argv) > 4 else "overlap"
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1")
    torch.cuda.set_device(0)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from speechrecognitionproject_amd import parallel
    # parallel.init_from_env leaves a 1-rank world alone: its RCCL settings by hand (device-bound group)
    parallel.nccl_env_for_graph_capture()
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    cap_group = parallel.capture_group()
    import importlib

    from oracle import models as OM
    from speechrecognitionproject_amd import _lib
    from speechrecognitionproject_amd import nn as snn
    from speechrecognitionproject_amd.graphs import GraphedStep
    from speechrecognitionproject_amd.optim import Adam, FlatParams
    from speechrecognitionproject_amd.synthetic import synthetic_clips

    ocls = {"mfcc_bgru": OM.MfccBGRU, "spec_bgru": OM.SpecBGRU, "resnet_bgru": OM.ResnetBGRU}[name]
    _lib.set_matmul_precision(precision)
    K = 3
    out = {}
    states = []
    for graphed in (False, True):
        torch.manual_seed(0)
        net = importlib.import_module("speechrecognitionproject_amd.models.model_" + name).Network().cuda()
        net.load_state_dict(OM.seeded_state_dict(ocls(), 0))
        net.train()
        if mode == "flat_syncbn":
            net = snn.convert_sync_batchnorm(net)
            snn.SyncBatchNorm1d.collectives_at_world1 = True
        flat = FlatParams(net.parameters())
        opt = Adam(net.parameters(), lr=1e-4, flat=flat)
        red = (parallel.GradReducer(flat, bucket_mb=0.5, collectives_at_world1=True, capture_group=cap_group)
               if mode == "overlap" else None)
        groups_used = []
        real_group_for_now = parallel.group_for_now

        def group_for_now(group=None, real=real_group_for_now):
            g = real(group)
            if torch.cuda.is_current_stream_capturing():
                groups_used.append(g is cap_group)
            return g
        parallel.group_for_now = group_for_now
        crit = snn.CrossEntropyLoss()
        # which stream the bucket launches see on their own thread (post-accumulate hooks run on
        # autograd's device thread): GradReducer issues them under the stream begin() saw either way
        hook_view = []
        if red is not None:
            orig_launch = red._launch

            def launch(i, orig=orig_launch):
                if red.capturing:
                    hook_view.append(bool(torch.cuda.is_current_stream_capturing()))
                orig(i)
            red._launch = launch
        x, y = synthetic_clips(3 * B, seed=23)
        pcm, lab = torch.from_numpy(x).cuda().view(3, B, -1), torch.from_numpy(y).cuda().view(3, B)
        sx, sy = pcm[0].clone(), lab[0].clone()
        launched = []

        def body():
            opt.zero_grad()
            if red is not None:
                red.begin()
            loss = crit(net(sx), sy)
            loss.backward()
            if red is not None:
                launched.append(len(red.works))          # collectives already forked during backward
                red.finish()
            else:
                parallel.allreduce_grads(flat, at_world1=True)
            opt.step()
            return loss

        losses = []
        if graphed:
            g = GraphedStep(body, warmup=2, capture_error_mode="thread_local")
            if red is not None:
                out["buckets"] = len(red.buckets)
                out["forked_during_backward"] = launched[-1]
                out["launch_thread_stream_capturing"] = hook_view
            out["captured_on_capture_group"] = groups_used
            for i in range(K):
                sx.copy_(pcm[(i + 1) % 3])
                sy.copy_(lab[(i + 1) % 3])
                losses.append(g.replay().item())
            g.release()
        else:
            for i in range(2 + K):
                if i >= 2:
                    sx.copy_(pcm[(i - 1) % 3])
                    sy.copy_(lab[(i - 1) % 3])
                loss = body()
                if i >= 2:
                    losses.append(loss.item())
        torch.cuda.synchronize()
        parallel.group_for_now = real_group_for_now
        snn.SyncBatchNorm1d.collectives_at_world1 = False
        if red is not None:
            red.remove()
        states.append((flat.data.clone(), opt.exp_avg.clone(), opt.exp_avg_sq.clone(), losses))
    (p0, m0, v0, l0), (p1, m1, v1, l1) = states
    out["losses_equal"] = l0 == l1
    out["params_equal"] = bool(torch.equal(p0, p1) and torch.equal(m0, m1) and torch.equal(v0, v1))
    out["spin_timeouts"] = _lib.spin_timeouts()

    # a captured collective runs on every replay: a 1-rank all-gather copies its input to its output.
    # An eager collective of the default group right before the capture (its Work still listed by the
    # watchdog) is the round-4 abort's precondition; the capture group keeps the two apart.
    src = torch.arange(1024, device="cuda", dtype=torch.float32)
    dst = torch.zeros(1024, device="cuda")
    dist.all_gather_into_tensor(dst, src)           # eager, default group
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        dist.all_gather_into_tensor(dst, src, group=cap_group)
    ok = []
    for r in range(3):
        src.fill_(r + 1.0)
        dst.zero_()
        g.replay()
        torch.cuda.synchronize()
        ok.append(bool(torch.all(dst == r + 1.0).item()))
    out["captured_collective_replays"] = ok

    # the abort's precondition, repeated: an eager collective of the default group (its Work listed by
    # the watchdog for up to its polling interval) immediately followed by a capture with a collective
    buf = torch.ones(1 << 16, device="cuda")
    sums = []
    for r in range(8):
        dist.all_reduce(buf)                         # eager, default group
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            dist.all_reduce(buf, group=cap_group)
            buf.add_(1.0)
        g.replay()
        torch.cuda.synchronize()
        sums.append(float(buf[0].item()))
    out["eager_then_capture"] = sums                 # 1-rank SUM is the identity: 2, 3, ..., 9
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
