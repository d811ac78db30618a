"""SDXL text encoders on the HIP path (encode_prompt, inference_animatediff.py:16-35) against
transformers' own CLIPTextModel / CLIPTextModelWithProjection -- the library the reference loads them with
(train_animatediff.py:74-80), importable here -- on the same weights and token ids.

No checkpoint or tokenizer vocabulary exists offline: weights are transformers' seeded random init of the two SDXL
text-tower configurations (rounded to bf16, the HIP path's weight precision, before both runs), token ids are a BOS,
random tokens, the EOS id (the largest id: SDXL's configs pool at argmax(ids), eos_token_id 2) and padding.  The
transformers run is fp32 (the reference's text encoders are fp32 modules); the yardstick is the same run under
torch.autocast(cuda, bf16), the reference's mixed precision.  Gate: within 1.25x of that yardstick (and 2e-2);
measured 0.9-1.04x (profiles/r3_text_encoder_gpu.log)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / b.norm()).item()


def _ids(B, vocab, pad, seed):
    g = torch.Generator().manual_seed(seed)
    ids = torch.full((B, 77), pad, dtype=torch.long)
    for b in range(B):
        n = 5 + 17 * b
        ids[b, 0] = vocab - 2                                        # <|startoftext|>
        ids[b, 1:n] = torch.randint(1, vocab - 2, (n - 1,), generator=g)
        ids[b, n] = vocab - 1                                        # <|endoftext|>: the largest id
    return ids


def _pair(cuda, which, with_proj):
    from transformers import CLIPTextConfig as TC
    from transformers import CLIPTextModel as TM
    from transformers import CLIPTextModelWithProjection as TMP
    from video_style_transfer_amd import text_encoder as T
    cfg = {"l": T.CLIPTextConfig.sdxl_text_encoder(), "g": T.CLIPTextConfig.sdxl_text_encoder_2(),
           "tiny": T.CLIPTextConfig.tiny("gelu")}[which]
    tc = TC(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size, intermediate_size=cfg.intermediate_size,
            num_hidden_layers=cfg.num_hidden_layers, num_attention_heads=cfg.num_attention_heads,
            max_position_embeddings=cfg.max_position_embeddings, hidden_act=cfg.hidden_act,
            layer_norm_eps=cfg.layer_norm_eps, projection_dim=cfg.projection_dim, eos_token_id=2,
            bos_token_id=cfg.vocab_size - 2, pad_token_id=1)
    torch.manual_seed(7)
    ref = (TMP if with_proj else TM)(tc).eval()
    with torch.no_grad():
        for p in ref.parameters():
            p.copy_(p.to(BF).float())  # the HIP path's bf16 weights, in both runs
    ref = ref.to(cuda)
    ours = T.build_text_encoder(T.CLIPTextModelWithProjection if with_proj else T.CLIPTextModel, cfg,
                                state_dict=ref.state_dict(), device=cuda)
    return cfg, ref, ours


@pytest.mark.parametrize("which,with_proj", [("tiny", True), ("l", False), ("g", True)])
def test_clip_text_encoder_vs_transformers(cuda, which, with_proj):
    cfg, ref, ours = _pair(cuda, which, with_proj)
    ids = _ids(2, cfg.vocab_size, cfg.vocab_size - 1 if which == "l" else 0, 3)
    tf32 = torch.backends.cuda.matmul.allow_tf32
    torch.backends.cuda.matmul.allow_tf32 = False
    try:
        with torch.no_grad():
            r = ref(ids.to(cuda), output_hidden_states=True)
            with torch.autocast("cuda", dtype=BF):
                y = ref(ids.to(cuda), output_hidden_states=True)
            o = ours(ids, output_hidden_states=True)
    finally:
        torch.backends.cuda.matmul.allow_tf32 = tf32
    pairs = [("hidden_states[-2]", o.hidden_states[-2], r.hidden_states[-2], y.hidden_states[-2]),
             ("last_hidden_state", o.last_hidden_state, r.last_hidden_state, y.last_hidden_state)]
    if with_proj:
        pairs.append(("text_embeds ([0])", o[0], r.text_embeds, y.text_embeds))
    assert len(o.hidden_states) == cfg.num_hidden_layers + 1
    for name, got, want, yard in pairs:
        e, ey = rel(got, want), rel(yard, want)
        print(f"[clip-{which}] {name}: HIP rel_l2 {e:.2e}; transformers bf16 autocast {ey:.2e}")
        assert got.shape == want.shape
        assert e <= 1.25 * ey and e <= 2e-2, (name, e, ey)


def test_encode_prompt_sdxl(cuda):
    """encode_prompt as the reference calls it: (1, 77, 768 + 1280) prompt embeddings from the penultimate layers,
    (1, 1280) pooled from text_encoder_2's projection; a stub tokenizer stands in for the CLIP BPE vocabulary."""
    from video_style_transfer_amd import text_encoder as T
    _, ref1, enc1 = _pair(cuda, "l", False)
    _, ref2, enc2 = _pair(cuda, "g", True)
    ids1, ids2 = _ids(1, 49408, 49407, 5), _ids(1, 49408, 0, 5)

    class Tok:
        model_max_length = 77

        def __init__(self, ids):
            self.ids = ids

        def __call__(self, prompt, **kw):
            assert kw["padding"] == "max_length" and kw["max_length"] == 77 and kw["truncation"]
            return type("T", (), {"input_ids": self.ids})()

    emb, pooled = T.encode_prompt(enc1, enc2, Tok(ids1), Tok(ids2), "a prompt", cuda)
    assert emb.shape == (1, 77, 2048) and pooled.shape == (1, 1280)
    with torch.no_grad():
        want = torch.cat([ref1(ids1.to(cuda), output_hidden_states=True).hidden_states[-2],
                          ref2(ids2.to(cuda), output_hidden_states=True).hidden_states[-2]], -1)
        wpool = ref2(ids2.to(cuda), output_hidden_states=True)[0]
    e, ep = rel(emb, want), rel(pooled, wpool)
    print(f"[encode_prompt] prompt_embeds rel_l2 {e:.2e}, pooled {ep:.2e}")
    assert e <= 2e-2 and ep <= 2e-2
