"""GPU: the HIP-graph decoder loop of the Tacotron (synthesizer/tacotron.py _generate_graph)
returns what the eager loop returns on the same device: same dropout masks (mask stream
advanced identically), same stop step, same stream position afterwards, and the same values
up to float rounding (under capture the BLAS library may pick other GEMM kernels: measured
differences are ~1e-6; bound 1e-4)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(stop_bias):
    from synthesizer.inference import build_tacotron
    from synthesizer.tacotron import synth_tacotron_state_dict
    m = build_tacotron('cpu')
    sd = synth_tacotron_state_dict(m, 7)
    sd['decoder.stop_proj.bias'] = torch.full_like(sd['decoder.stop_proj.bias'], stop_bias)
    m.load_state_dict(sd)
    return m.cuda().eval()


@pytest.mark.parametrize('stop_bias,steps', [(-8.0, 70), (8.0, 200)])
def test_graph_decoder_equals_eager(stop_bias, steps):
    from synthesizer.tacotron import set_dropout_stream
    import synthesizer.tacotron as tc
    m = _model(stop_bias)
    rng = np.random.default_rng(4)
    chars = torch.from_numpy(rng.integers(1, 60, (2, 23))).cuda()  # symbol ids (66 symbols)
    chars[1, 17:] = 0
    spk = torch.from_numpy(rng.normal(size=(2, 768)).astype(np.float32)).cuda()
    out = {}
    for graph in (False, True):
        set_dropout_stream(11)
        out[graph] = [t.cpu().numpy() for t in m.generate(chars, spk, steps=steps, graph=graph)]
        out[graph].append(tc._dropout.calls)
    set_dropout_stream(None)
    e, g = out[False], out[True]
    assert e[0].shape == g[0].shape
    if stop_bias > 0:  # stops at the first allowed step (t > 10), inside the first chunk
        assert e[0].shape[2] == 12
    for a, b in zip(e[:3], g[:3]):
        assert np.abs(a - b).max() < 1e-4
    assert e[3] == g[3]
