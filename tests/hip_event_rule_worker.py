"""Worker of tests/test_dp_graph_gpu.py::test_hip_rule_event_on_stream_joined_to_capture (a subprocess:
a failed query inside a capture must not disturb the test process).

The rule under test (the round-4 watchdog abort): an event recorded EAGERLY on stream S,
its work long finished, is queried from another thread (as ProcessGroupNCCL's watchdog does) while S
has been joined to a capture running on another stream C (S waited on an event recorded in the
capture, which is what a collective issued during a capture does to the process group's stream).
Control: the same query while a capture runs that S never joins.  Prints one JSON line."""
import json
import threading

import torch


def query_in_thread(ev):
    out = {}

    def run():
        try:
            out["done"] = bool(ev.query())
        except RuntimeError as e:   # torch raises the HIP error of hipEventQuery
            out["error"] = str(e).splitlines()[0]

    t = threading.Thread(target=run)
    t.start()
    t.join()
    return out


def main():
    torch.cuda.set_device(0)
    S, C = torch.cuda.Stream(), torch.cuda.Stream()
    x = torch.zeros(1 << 20, device="cuda")
    e = torch.cuda.Event()
    with torch.cuda.stream(S):
        x.add_(1.0)
        e.record(S)
    torch.cuda.synchronize()
    res = {"eager_before": query_in_thread(e)}

    # control: a capture on C that S never joins
    g0 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g0, stream=C, capture_error_mode="relaxed"):
        x.add_(0.5)
        res["capture_not_joined"] = query_in_thread(e)

    # S joins the capture through an event recorded in it, then is joined back before it ends
    g1 = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g1, stream=C, capture_error_mode="relaxed"):
            f = torch.cuda.Event()
            f.record(C)
            S.wait_event(f)
            res["S_joined"] = query_in_thread(e)
            try:
                with torch.cuda.stream(S):
                    x.add_(1.0)
                res["capture_after_query"] = "ok"
            except RuntimeError as err:
                res["capture_after_query"] = str(err).splitlines()[0]
            C.wait_stream(S)
        res["capture_end"] = "ok"
    except RuntimeError as err:
        res["capture_end"] = str(err).splitlines()[0]
    torch.cuda.synchronize()
    res["after_capture"] = query_in_thread(e)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
