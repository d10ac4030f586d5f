"""wav2vec2's positional-conv weight norm as a plain reduction (vdiff.unet_audio.
_swap_weight_norm) against torch's own parametrization: same weight, output and gradients,
same state-dict keys.  CPU."""
import copy

import torch

from vdiff.unet_audio import _WeightNormReduce, _swap_weight_norm


def test_swapped_weight_norm_matches_torch():
    from transformers import Wav2Vec2Config, Wav2Vec2Model
    torch.manual_seed(0)
    ref = Wav2Vec2Model(Wav2Vec2Config(num_hidden_layers=1, hidden_size=96, intermediate_size=128,
                                       num_attention_heads=4, num_conv_pos_embeddings=16,
                                       num_conv_pos_embedding_groups=4)).eval()
    new = copy.deepcopy(ref)
    _swap_weight_norm(new)
    conv = new.encoder.pos_conv_embed.conv
    assert isinstance(conv.parametrizations.weight[0], _WeightNormReduce)
    assert list(new.state_dict()) == list(ref.state_dict())
    torch.testing.assert_close(conv.weight, ref.encoder.pos_conv_embed.conv.weight,
                               rtol=1e-6, atol=1e-7)
    x = torch.randn(2, 2000)
    a, b = ref(x).last_hidden_state, new(x).last_hidden_state
    torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-5)
    a.square().sum().backward()
    b.square().sum().backward()
    # fp64 reference gradients: the first feature-extractor conv's gradient is ill-conditioned
    # (fp32 torch itself is 13 % off fp64 there), so each fp32 gradient is judged against
    # fp64 and the swapped model may not be worse than torch's own fp32 by more than 1e-5
    r64 = copy.deepcopy(ref).double()
    r64.zero_grad()
    r64(x.double()).last_hidden_state.square().sum().backward()
    for (n1, p1), (n2, p2), (_, p3) in zip(ref.named_parameters(), new.named_parameters(),
                                           r64.named_parameters()):
        assert n1 == n2
        assert (p1.grad is None) == (p2.grad is None), n1
        if p1.grad is None:  # e.g. the masked-time-step embedding (unused without a mask)
            continue
        scale = p3.grad.norm().clamp_min(1e-30)
        e_ref = ((p1.grad.double() - p3.grad).norm() / scale).item()
        e_new = ((p2.grad.double() - p3.grad).norm() / scale).item()
        assert e_new <= 1.5 * e_ref + 1e-5, (n1, e_new, e_ref)


def test_spec_augment_mask_without_index_put_matches_transformers():
    """Train-mode SpecAugment (time and feature masks) through vdiff's torch.where form
    against transformers' boolean index_put: same numpy draws, same output and gradients."""
    import numpy as np
    import types
    from transformers import Wav2Vec2Config, Wav2Vec2Model
    from vdiff.unet_audio import _mask_hidden_states
    torch.manual_seed(0)
    cfg = Wav2Vec2Config(num_hidden_layers=1, hidden_size=96, intermediate_size=128,
                         num_attention_heads=4, num_conv_pos_embeddings=16,
                         num_conv_pos_embedding_groups=4, mask_time_prob=0.6, mask_time_length=2,
                         mask_feature_prob=0.3, mask_feature_length=4, layerdrop=0.0,
                         hidden_dropout=0.0, attention_dropout=0.0, activation_dropout=0.0,
                         feat_proj_dropout=0.0)
    ref = Wav2Vec2Model(cfg).train()
    new = copy.deepcopy(ref)
    new._mask_hidden_states = types.MethodType(_mask_hidden_states, new)
    x = torch.randn(3, 4000)
    outs = []
    for m in (ref, new):
        np.random.seed(7)
        out = m(x).last_hidden_state
        out.square().sum().backward()
        outs.append(out)
    torch.testing.assert_close(outs[1], outs[0], rtol=0, atol=0)
    for (n1, p1), (_, p2) in zip(ref.named_parameters(), new.named_parameters()):
        if p1.grad is None:
            assert p2.grad is None, n1
            continue
        torch.testing.assert_close(p2.grad, p1.grad, rtol=1e-5, atol=1e-7), n1
    assert ref.masked_spec_embed.grad.abs().sum() > 0  # the time mask was applied
