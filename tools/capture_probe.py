"""Capture-topology probe for the hipStreamEndCapture segfault.

Each variant captures a small graph with torch.cuda.graph on the model's pooled-event
forks (vt_stream_fork / vt_stream_mark) and reports OK or the Python exception; a
segfault ends the process (the caller runs one variant per process and stops at the
first crash, as the GPU-box rules require).

  python tools/capture_probe.py VARIANT
    fork_join        main -> s3 fork, kernel on s3, join            (the model's pattern)
    eager_then_fork  s3 used eagerly first, then forked in the capture
    reuse_branch     s1 forked, joined, then forked again for a second branch
    external_wait    wait inside the capture on a pooled event recorded OUTSIDE it
    unjoined         s3 forked and never joined before capture_end
    model_branches   the S=16 model step with the head / LSTM weight-gradient branches kept
                     under capture (VAETEB_CAPTURE_BRANCHES=1, set by this script)
    model_head       ... the head weight-gradient branch only (side stream 1)
    model_lstm       ... the LSTM weight-gradient branch only (side stream 2)
    model_head_norec ... the head branch with Tensor.record_stream disabled
    model_head_join  ... the head branch joined back to the main stream right after its kernel
    model_head_info  ... model_head with the capture state dumped (VAETEB_CAPTURE_TRACE)
    model_lstm_info  ... model_lstm with the capture state dumped (the branch that captures fine)
    unjoined_refork  s1 forked, kernel, NOT joined, forked again, kernel, joined (the head
                     branch's shape: side stream 1 is forked again by the encoders' backward)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "vae-teb_amd"), os.path.join(ROOT, "tests")]
variant = sys.argv[1]
if variant.startswith("model_"):
    os.environ["VAETEB_CAPTURE_BRANCHES"] = "1"
    # model_branches: both branches; model_head: the head weight gradients on side stream 1 only
    # (the production setting, dropped under capture); model_lstm: the LSTM weight gradients on
    # side stream 2 only
    os.environ["VAETEB_LSTM_GRAD_SIDE_STREAM"] = "0" if variant.startswith("model_head") else "2"
    os.environ["VAETEB_HEAD_GRAD_SIDE_STREAM"] = "0" if variant.startswith("model_lstm") else "1"
    if variant == "model_head_join":
        os.environ["VAETEB_HEAD_GRAD_JOIN"] = "1"
    if variant in ("model_head_info", "model_lstm_info"):
        # round 6: the capture state (hipStreamGetCaptureInfo_v2, node types,
        # dependency sets) of the side stream right after the head branch and of every stream
        # before the capture ends, printed to stderr (vaeteb._lib.capture_info)
        os.environ["VAETEB_CAPTURE_TRACE"] = "1"

import torch  # noqa: E402

from vaeteb import _lib  # noqa: E402

if variant == "model_head_norec":
    # the head branch without Tensor.record_stream (the allocator's cross-stream use
    # tracking under capture): isolates it as the trigger
    torch.Tensor.record_stream = lambda self, stream: None


def kern(t, s=None):
    """one small kernel on the current (or given) stream: t += 1 via the library's vt_scale kernel"""
    with torch.cuda.stream(s) if s is not None else torch.cuda.stream(torch.cuda.current_stream()):
        t.add_(1.0)


def run():
    dev = torch.device("cuda:0")
    a = torch.zeros(1 << 16, device=dev)
    b = torch.zeros(1 << 16, device=dev)
    s1, s3 = torch.cuda.Stream(), torch.cuda.Stream()
    if variant.startswith("model_"):
        import numpy as np
        from golden_util import det_fill_
        from vaeteb.model import SeqVaeTeb
        from vaeteb.train import Trainer
        g = np.load(os.path.join(ROOT, "tests", "golden", "model_s16_b4.npz"), allow_pickle=False)
        T = lambda k: torch.from_numpy(g[k]).cuda()
        batch = {"fhr_st": T("y_st"), "fhr_ph": T("y_ph"), "fhr_up_ph": T("x_ph"), "fhr": T("y_raw")}
        m = det_fill_(SeqVaeTeb(sequence_length=16, concurrent_encoders=True, head_precision="bf16",
                                conv_precision="bf16", mlp_precision="bf16")).cuda()
        tr = Trainer(m, lr=1e-3)
        cap = tr.capture(batch, eps=T("eps"), warmup=2, native=True)
        print("captured; replay loss", cap.replay(batch, eps=T("eps"))["total_loss"].item())
        return
    if variant == "eager_then_fork":
        kern(b, s3)
        slot = _lib.mark(s3)
        _lib.wait_mark(slot)
        torch.cuda.synchronize()
    ext_slot = None
    if variant == "external_wait":
        kern(b, s3)
        ext_slot = _lib.mark(s3)
    graph = torch.cuda.CUDAGraph()
    cap_stream = torch.cuda.Stream()
    cap_stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cap_stream):
        with torch.cuda.graph(graph, stream=cap_stream):
            kern(a)
            if variant in ("fork_join", "eager_then_fork", "unjoined"):
                _lib.wait_for(s3)                       # s3 waits on the capture stream
                kern(b, s3)
                if variant != "unjoined":
                    _lib.wait_for(torch.cuda.current_stream(), s3)
            elif variant == "reuse_branch":
                for _ in range(2):
                    _lib.wait_for(s1)
                    kern(b, s1)
                    _lib.wait_for(torch.cuda.current_stream(), s1)
                    kern(a)
            elif variant == "unjoined_refork":
                _lib.wait_for(s1)
                kern(b, s1)                              # left unjoined
                kern(a)
                _lib.wait_for(s1)                        # forked again
                kern(b, s1)
                _lib.wait_for(torch.cuda.current_stream(), s1)
            elif variant == "external_wait":
                _lib.wait_mark(ext_slot)
                kern(a)
            kern(a)
    graph.replay()
    torch.cuda.synchronize()
    print("replayed", a[0].item(), b[0].item())


if __name__ == "__main__":
    try:
        run()
        print(f"VARIANT {variant}: OK", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"VARIANT {variant}: {type(e).__name__}: {e}", flush=True)
