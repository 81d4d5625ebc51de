"""Config-4 classifier: host-side contract checks that need no GPU — the HIP
modules carry the reference's state_dict keys in the reference's order
(checkpoint interchange with ref/model/inception_time.py and
ref/model/vae_teb_model.py:1248-1526) and the constructor arguments mirror it."""
import numpy as np


def test_classifier_state_dict_keys_match_reference(golden):
    from oracle import classifier_ref as C
    from vaeteb.classifier import FHRInceptionTimeClassifier
    g = golden("classifier_s64_b4")
    m = FHRInceptionTimeClassifier()
    assert [k for k, _ in m.named_parameters()] == list(g["param_names"])
    ref = C.InceptionTimeClassifier()
    assert list(m.state_dict().keys()) == list(ref.state_dict().keys())
    for k, v in ref.state_dict().items():
        assert tuple(m.state_dict()[k].shape) == tuple(v.shape), k
    assert list(g["bn_names"]) == [k for k in m.state_dict() if k.endswith(("running_mean", "running_var"))]


def test_seqvae_classifier_keys(golden):
    from vaeteb.classifier import SeqVaeTebClassifier
    g = golden("seqvae_classifier_s16_b4")
    m = SeqVaeTebClassifier(sequence_length=16, freeze_vae=False)
    assert [k for k, _ in m.named_parameters()] == list(g["param_names"])
    frozen = SeqVaeTebClassifier(sequence_length=16, freeze_vae=True)
    assert not any(p.requires_grad for p in frozen.vae_model.parameters())
    assert all(p.requires_grad for p in frozen.classifier.parameters())
    assert np.isfinite(g["total_loss"])
