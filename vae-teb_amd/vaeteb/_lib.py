"""ctypes binding of libvaeteb.so (the C ABI declared in include/vaeteb.h).

Signatures are read from the header itself, so the Python side can never drift
from the C side.  There is deliberately NO fallback: if the shared library is
missing or was built for another architecture, importing any op raises, and the
training step does not silently run on PyTorch kernels instead.
"""
import ctypes
import os
import re

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(os.path.dirname(_HERE))
LIB_PATH = os.environ.get("VAETEB_LIB", os.path.join(_HERE, "_lib", "libvaeteb.so"))
HEADER = os.path.join(_ROOT, "include", "vaeteb.h")

VT_ERR_ARG, VT_ERR_LAYOUT, VT_ERR_HIP = -1, -2, -3

_CT = {
    "int": ctypes.c_int, "int64_t": ctypes.c_int64, "float": ctypes.c_float, "double": ctypes.c_double,
    "void*": ctypes.c_void_p, "float*": ctypes.c_void_p, "double*": ctypes.c_void_p, "int*": ctypes.c_void_p, "int64_t*": ctypes.c_void_p,
    "char*": ctypes.c_char_p,
}


def parse_header(path=HEADER):
    """Return {name: (restype_str, [arg_type_str, ...])} for every `vt_*` prototype."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", " ", src, flags=re.S)
    protos = {}
    for m in re.finditer(r"\b(const\s+char\s*\*|int|void)\s+(vt_\w+)\s*\(([^)]*)\)\s*;", src):
        ret, name, args = m.group(1).replace(" ", ""), m.group(2), m.group(3).strip()
        types = []
        if args and args != "void":
            for a in args.split(","):
                a = a.replace("const", " ").strip()
                a = re.sub(r"\s*\*\s*", "* ", a)
                a = re.sub(r"\b\w+$", "", a.strip()).strip()  # drop the parameter name
                a = a.replace(" ", "")
                if a.endswith("**") or a.endswith("*const*"):
                    a = "void*"
                types.append(a)
        protos[name] = (ret, types)
    return protos


class VtError(RuntimeError):
    pass


class _Lib:
    def __init__(self):
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libvaeteb.so not found at {LIB_PATH}. Build it first: "
                f"`python -c 'import __graft_entry__ as g; g.build()'` (or `make -C vae-teb_amd/csrc`).")
        self.dll = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        self.protos = parse_header()
        self.fns = {}
        for name, (ret, args) in self.protos.items():
            f = getattr(self.dll, name)
            f.restype = ctypes.c_char_p if ret == "constchar*" else ctypes.c_int
            f.argtypes = [_CT[a] for a in args]
            self.fns[name] = f
        # DIAGNOSTIC ONLY (tools/ablate_step.sh): VAETEB_ABLATE=name[,name...] turns the named
        # entry points into no-ops, so a timing run shows how much of the step a kernel
        # family holds on the critical path.  Results are then wrong; never set in training.
        ablate = [n for n in os.environ.get("VAETEB_ABLATE", "").split(",") if n]
        for n in ablate:
            if n not in self.fns:
                raise KeyError(f"VAETEB_ABLATE: unknown entry point {n}")
            self.fns[n] = lambda *a: 0
        # A/B switch of the bf16 conv kernels (vt_conv_bf16_set_kernels; same bits either way)
        if "VAETEB_CONV_KERNELS" in os.environ:
            self.call("vt_conv_bf16_set_kernels", int(os.environ["VAETEB_CONV_KERNELS"]))

    def last_error(self):
        return self.fns["vt_last_error"]().decode()

    def call(self, name, *args):
        rc = self.fns[name](*args)
        if rc != 0:
            msg = f"{name}: {self.last_error()}"
            if rc == VT_ERR_ARG:
                raise ValueError(msg)
            raise VtError(msg)
        return rc


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _Lib()
    return _lib


def ptr(t):
    """Device pointer of a tensor (None -> NULL).  Tensors must be contiguous."""
    if t is None:
        return None
    if not t.is_contiguous():
        raise RuntimeError("Tensors must be contiguous.")
    return t.data_ptr()


def stream():
    """Raw handle of the current HIP stream (~0.3 us; torch.cuda.current_stream()
    builds a Python Stream object per call, ~2.6 us)."""
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def call(name, *args):
    return lib().call(name, *args)


def wait_for(waiter, src=None):
    """Stream `waiter` waits for the work enqueued so far on `src` (default: the
    current stream) — torch's `waiter.wait_stream(src)` through the library's
    pooled events (vt_stream_fork), without a Python Event per fork."""
    w = waiter if isinstance(waiter, int) else waiter.cuda_stream
    s = stream() if src is None else (src if isinstance(src, int) else src.cuda_stream)
    if w != s:
        rc = lib().fns["vt_stream_fork"](s, w)
        if rc != 0:
            raise RuntimeError(f"vt_stream_fork: {lib().last_error()}")


_H16 = [None]


def set_h16(fp16):
    """The library's 16-bit MFMA operand format (vt_set_h16_format): False bf16 (default), True fp16
    (the reference's autocast width, trained with a dynamic loss scale: vaeteb.train.Trainer)."""
    v = 1 if fp16 else 0
    if _H16[0] != v:
        lib().fns["vt_set_h16_format"](v)
        _H16[0] = v


def h16():
    """The current 16-bit operand format: 'fp16' or 'bf16'."""
    return "fp16" if lib().fns["vt_get_h16_format"]() else "bf16"


def capture_info(src=None):
    """Diagnostic: the hipGraph capture state of stream `src` (default: the current stream) as
    text — vt_capture_info (tools/capture_probe.py)."""
    import ctypes
    buf = ctypes.create_string_buffer(1 << 16)
    s = stream() if src is None else (src if isinstance(src, int) else src.cuda_stream)
    call("vt_capture_info", s, buf, len(buf))
    return buf.value.decode()


def mark(src=None):
    """A pooled event recorded on `src` (default: the current stream); see wait_mark."""
    import ctypes
    slot = ctypes.c_int()
    call("vt_stream_mark", stream() if src is None else src.cuda_stream, ctypes.byref(slot))
    return slot.value


def wait_mark(slot, waiter=None):
    """`waiter` (default: the current stream) waits for the point `mark` recorded."""
    call("vt_stream_wait_mark", stream() if waiter is None else waiter.cuda_stream, slot)
