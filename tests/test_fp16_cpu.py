"""Host logic of the fp16 operand format (round 6), CPU only: the model's precision setters keep
one 16-bit format per model and flag loss scaling exactly for fp16; the trainer defaults its
dynamic loss scale from it (GradScaler('cuda') in the reference's fp16 loop,
ref/model/graph_model.py:670).  The kernels themselves: tests/test_gpu_fp16.py."""
import pytest

from vaeteb import ops
from vaeteb.model import SeqVaeTeb


def test_h16_flag_normalisation():
    assert ops.h16_flag(False) is False and ops.h16_flag(None) is False
    assert ops.h16_flag(True) == "bf16" and ops.h16_flag("bf16") == "bf16"
    assert ops.h16_flag("fp16") == "fp16"


@pytest.mark.parametrize("prec,fmt,scaled", [("fp32", None, False), ("bf16", "bf16", False), ("fp16", "fp16", True)])
def test_model_format_and_loss_scaling(prec, fmt, scaled):
    m = SeqVaeTeb(sequence_length=16, head_precision=prec, conv_precision=prec, mlp_precision=prec)
    assert m.h16_format == fmt and m.loss_scaling == scaled
    flags = {getattr(mod, "bf16") for mod in m.modules() if type(mod).__name__ in ("ResidualMLP", "ConvBlock")}
    assert flags == {False if prec == "fp32" else prec}
    heads = {mod.mfma for h in (m.decoder.output_mu, m.decoder.output_logvar) for mod in h.modules()
             if hasattr(mod, "mfma")}
    assert heads == {False if prec == "fp32" else prec}


def test_mixed_16bit_formats_rejected():
    with pytest.raises(ValueError, match="mix bf16 and fp16"):
        SeqVaeTeb(sequence_length=16, head_precision="fp16", conv_precision="bf16", mlp_precision="fp16")
    m = SeqVaeTeb(sequence_length=16, head_precision="fp16", conv_precision="fp16", mlp_precision="fp32")
    assert m.loss_scaling
    with pytest.raises(ValueError):
        m.set_mlp_precision("bf16")
    with pytest.raises(ValueError):
        m.set_head_precision("fp8")
