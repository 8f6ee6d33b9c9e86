"""Tokenizers (SentencePiece / tiktoken-format BPE with the C++ merge core), Meta checkpoint
conversion with 1/2/4 shards, partition rules, and the string-level LLaMA generator API.

Reference behaviour: llama2_tokenizer.py:14-71, llama3_tokenizer.py:38-232 (ChatFormat :205-232),
convert_weights.py:52-92, partition.py:10-98, generation.py:47-79. Tiny models are trained /
written locally (no network): tokenizer parity vs Meta's real files is "parity unpinned".
"""
from __future__ import annotations

import base64
import collections
import json
import os

import pytest
import torch

from jax_llama_amd import (LLaMA, LLaMA2Tokenizer, LLaMA3Tokenizer, ChatFormat, convert_llama_weights,
                           get_llama_param_partition_spec)
from jax_llama_amd.parallel.partition import P, Mesh, shard_tree, with_named_sharding_constraint
from jax_llama_amd.tokenizer.bpe import PyBPE, load_tiktoken_bpe, save_tiktoken_bpe
from jax_llama_amd.utils.checkpoint import (meta_state_dict_to_params, params_json_for, random_meta_state_dict,
                                            save_meta_checkpoint)
from helpers import build, tiny_config

CORPUS = ("The quick brown fox jumps over the lazy dog. LLaMA runs on MI355X with HIP kernels!\n"
          "Numbers 12345 and 678, unicode café naïve 日本語, tabs\tand  spaces.  ") * 20


# ------------------------------------------------------------------ tokenizers
def _train_bpe_ranks(text: str, n_merges: int = 150):
    """Tiny byte-level BPE trainer -> tiktoken-style {bytes: rank}."""
    ranks = {bytes([i]): i for i in range(256)}
    words = [list(bytes([b]) for b in w.encode()) for w in text.split(" ")]
    for _ in range(n_merges):
        pairs = collections.Counter()
        for w in words:
            for a, b in zip(w, w[1:]):
                pairs[(a, b)] += 1
        if not pairs:
            break
        (a, b), _ = pairs.most_common(1)[0]
        ranks[a + b] = len(ranks)
        new_words = []
        for w in words:
            out, i = [], 0
            while i < len(w):
                if i + 1 < len(w) and w[i] == a and w[i + 1] == b:
                    out.append(a + b)
                    i += 2
                else:
                    out.append(w[i])
                    i += 1
            new_words.append(out)
        words = new_words
    return ranks


@pytest.fixture(scope="module")
def llama3_tok(tmp_path_factory):
    path = str(tmp_path_factory.mktemp("tok") / "tokenizer.model")
    save_tiktoken_bpe(_train_bpe_ranks(CORPUS), path)
    return LLaMA3Tokenizer(path)


def test_tiktoken_file_roundtrip(tmp_path):
    ranks = _train_bpe_ranks(CORPUS, 40)
    p = str(tmp_path / "r.model")
    save_tiktoken_bpe(ranks, p)
    assert load_tiktoken_bpe(p) == ranks
    line = open(p).readline().split()
    assert base64.b64decode(line[0]) in ranks


def test_llama3_encode_decode_roundtrip(llama3_tok):
    tok = llama3_tok
    for s in ["hello world", CORPUS[:300], "日本語 café", "", "   ", "a\n\nb\r\n c"]:
        ids = tok.encode(s, bos=True, eos=True)
        assert ids[0] == tok.bos_id and ids[-1] == tok.eos_id
        assert tok.decode(ids[1:-1]) == s
    assert len(tok) == tok.n_words == len(tok.model.mergeable_ranks) + tok.num_reserved_special_tokens
    assert tok.pad_id == -1
    assert tok.stop_tokens == {tok.eos_id, tok.special_tokens["<|eot_id|>"]}


def test_native_bpe_matches_python_reference(llama3_tok):
    tok = llama3_tok
    if not tok.model.native:
        pytest.skip("native BPE core not built")
    ranks = {k: v for k, v in tok.model.mergeable_ranks.items()}
    py = PyBPE(ranks)
    import regex
    pieces = [m.encode() for m in regex.findall(tok.pat_str, CORPUS[:2000])]
    assert tok.model.encode_ordinary(CORPUS[:2000]) == py.encode_pieces(pieces)


def test_special_tokens_and_chat_format(llama3_tok):
    tok = llama3_tok
    s = "<|begin_of_text|>hi"
    with pytest.raises(ValueError):
        tok.encode(s, bos=False, eos=False, disallowed_special="all")
    ids = tok.encode(s, bos=False, eos=False, allowed_special="all")
    assert ids[0] == tok.bos_id
    ids2 = tok.encode(s, bos=False, eos=False, disallowed_special=())
    assert tok.bos_id not in ids2 and tok.decode(ids2) == s
    fmt = ChatFormat(tok)
    dialog = [{"role": "system", "content": "be brief"}, {"role": "user", "content": "hello"}]
    ids = fmt.encode_dialog_prompt(dialog)
    sh, eh, eot = (tok.special_tokens[k] for k in ("<|start_header_id|>", "<|end_header_id|>", "<|eot_id|>"))
    assert ids[0] == tok.bos_id
    assert ids.count(sh) == 3 and ids.count(eh) == 3 and ids.count(eot) == 2
    assert tok.decode(ids).endswith("<|start_header_id|>assistant<|end_header_id|>\n\n")


def test_long_whitespace_chunking(llama3_tok):
    s = " " * 30000 + "x" * 30000
    ids = llama3_tok.encode(s, bos=False, eos=False)
    assert llama3_tok.decode(ids) == s


def _pieces_oracle(s, window, max_run):
    """Chunking semantics of the reference tokenizer (llama3_tokenizer.py:131-146,178-202), written as a
    per-character state machine: a new piece starts at every window start and whenever a same-class
    run has reached max_run characters."""
    out = []
    for w0 in range(0, max(len(s), 1), window):
        win = s[w0:w0 + window]
        piece, run, prev = "", 0, None
        for ch in win:
            cls = ch.isspace()
            run = run + 1 if cls == prev else 1
            if run > max_run:
                out.append(piece)
                piece, run = "", 1
            piece += ch
            prev = cls
        out.append(piece)
    return [p for p in out if p]


def test_chunk_bounds_native_python_oracle():
    from jax_llama_amd.tokenizer.llama3 import _chunk_bounds_py, chunk_bounds
    import random
    rnd = random.Random(0)
    alphabet = [" ", "\t", "\n", "a", "b", "\u3000", "\xa0", "\u2003", "\u200b", "1", "\x1c"]
    for _ in range(300):
        s = "".join(rnd.choice(alphabet) * rnd.randint(1, 9) for _ in range(rnd.randint(0, 12)))
        window, run = rnd.randint(1, 40), rnd.randint(1, 12)
        for fn in (chunk_bounds, _chunk_bounds_py):
            b = fn(s, window, run)
            assert [s[lo:hi] for lo, hi in zip(b, b[1:]) if hi > lo] == _pieces_oracle(s, window, run), (s, window, run)


@pytest.fixture(scope="module")
def sp_tok(tmp_path_factory):
    spm = pytest.importorskip("sentencepiece")
    d = tmp_path_factory.mktemp("sp")
    corpus = d / "corpus.txt"
    corpus.write_text(CORPUS.replace(". ", ".\n"))
    spm.SentencePieceTrainer.train(input=str(corpus), model_prefix=str(d / "m"), vocab_size=120,
                                   model_type="bpe", bos_id=1, eos_id=2, pad_id=-1, unk_id=0,
                                   minloglevel=2)
    return LLaMA2Tokenizer(str(d / "m.model"))


def test_llama2_tokenizer(sp_tok):
    ids = sp_tok.encode("The quick brown fox", bos=True, eos=False)
    assert ids[0] == sp_tok.bos_id == 1 and sp_tok.eos_id == 2 and sp_tok.pad_id == -1
    assert sp_tok.decode(ids[1:]) == "The quick brown fox"
    assert len(sp_tok) == sp_tok.n_words == 120


# ------------------------------------------------------------------ checkpoint conversion
@pytest.mark.parametrize("n_shards,vocab_parallel", [(1, False), (2, False), (4, False), (2, True), (8, False)])
def test_convert_meta_checkpoint(tmp_path, n_shards, vocab_parallel):
    # (8, False): the LLaMA-1 65B layout -- 8 consolidated.XX.pth shards, ParallelEmbedding split on the
    # model dim (BASELINE.json config 5, download.sh:10-13)
    cfg = tiny_config(num_attention_heads=8, num_key_value_heads=8, intermediate_size=96)
    sd = random_meta_state_dict(cfg, seed=5)
    pj = params_json_for(cfg, multiple_of=32)
    pj["some_future_key"] = 1  # unknown params.json keys are tolerated (reference ModelArgs rejects)
    save_meta_checkpoint(sd, pj, str(tmp_path), n_shards=n_shards, vocab_parallel_embedding=vocab_parallel)
    params, config = convert_llama_weights(str(tmp_path), cfg.vocab_size, max_seq_len=64)
    assert config.hidden_size == cfg.hidden_size and config.num_key_value_heads == 8
    assert config.intermediate_size == 96 and config.vocab_size == cfg.vocab_size
    assert config.max_sequence_length == 64
    want = meta_state_dict_to_params(sd, cfg.num_hidden_layers)
    flat_a = json.dumps(sorted(_flat(params)))
    assert flat_a == json.dumps(sorted(_flat(want)))
    for k, v in _flat_items(want):
        got = _get(params, k)
        assert torch.equal(torch.as_tensor(got).to(v.dtype), torch.as_tensor(v)), k


@pytest.mark.parametrize("n_shards,tp", [(1, 2), (2, 2), (4, 2), (2, 4), (4, 1), (2, 1), (8, 8), (8, 2), (1, 8)])
def test_load_meta_rank_equals_sharded_merge(tmp_path, n_shards, tp):
    # (8, 8): LLaMA-1 65B at MP=8 from its 8-shard checkpoint, every rank reading only its own slices
    from jax_llama_amd.utils.checkpoint import load_meta_rank
    cfg = tiny_config(num_attention_heads=8, num_key_value_heads=8, intermediate_size=96)
    sd = random_meta_state_dict(cfg, seed=6)
    save_meta_checkpoint(sd, params_json_for(cfg, multiple_of=32), str(tmp_path), n_shards=n_shards,
                         vocab_parallel_embedding=(n_shards == 4))
    full, _ = convert_llama_weights(str(tmp_path), cfg.vocab_size, max_seq_len=64)
    for r in range(tp):
        got, config = load_meta_rank(str(tmp_path), cfg.vocab_size, r, tp, max_seq_len=64, dtype=None)
        want = shard_tree(full, r, tp)
        for k, v in _flat_items(want):
            g = torch.as_tensor(_get(got, k))
            assert g.shape == torch.as_tensor(v).shape, k
            assert torch.equal(g, torch.as_tensor(v)), k


def _flat(t, pre=()):
    out = []
    for k, v in t.items():
        out += _flat(v, pre + (k,)) if isinstance(v, dict) else ["/".join(pre + (k,))]
    return out


def _flat_items(t, pre=()):
    for k, v in t.items():
        if isinstance(v, dict):
            yield from _flat_items(v, pre + (k,))
        else:
            yield "/".join(pre + (k,)), v


def _get(t, path):
    for k in path.split("/"):
        t = t[k]
    return t


def test_ffn_size_formula_matches_meta():
    from jax_llama_amd.config import swiglu_hidden_size, get_preset
    assert swiglu_hidden_size(4096, 256) == 11008          # LLaMA 7B
    assert swiglu_hidden_size(5120, 256) == 13824          # 13B
    assert swiglu_hidden_size(8192, 4096, 1.3) == 28672    # Llama-2/3 70B
    assert swiglu_hidden_size(4096, 1024, 1.3) == 14336    # Llama-3 8B
    assert get_preset("8b").intermediate_size == 14336


# ------------------------------------------------------------------ partition rules
def test_partition_spec_complete_and_shards():
    cfg = tiny_config()
    _, _, _, params = build(cfg)
    spec = get_llama_param_partition_spec(params)
    assert spec["transformer"]["h"]["0"]["attention"]["wq"]["kernel"] == P(None, "mp")
    assert spec["transformer"]["h"]["0"]["attention"]["wo"]["kernel"] == P("mp", None)
    assert spec["lm_head"]["kernel"] == P(None, "mp")
    fs = get_llama_param_partition_spec(params, fsdp=True)
    assert fs["transformer"]["h"]["0"]["feed_forward"]["w2"]["kernel"] == P("mp", "dp")
    sh = shard_tree(params, 1, 2)
    wq = torch.as_tensor(params["transformer"]["h"]["0"]["attention"]["wq"]["kernel"])
    assert torch.equal(torch.as_tensor(sh["transformer"]["h"]["0"]["attention"]["wq"]["kernel"]),
                       wq[:, wq.shape[1] // 2:])
    with pytest.raises(AssertionError):
        from jax_llama_amd.parallel.partition import get_partition_spec
        get_partition_spec({"mystery": {"kernel": 1}}, [])


def test_named_sharding_constraint_splits_batch():
    x = torch.arange(8).reshape(4, 2)
    assert torch.equal(with_named_sharding_constraint(x, None, P("dp", None)), x)
    m = Mesh(dp=2, mp=1, rank=1)
    assert torch.equal(with_named_sharding_constraint(x, m, P("dp", None)), x[2:])


# ------------------------------------------------------------------ string-level generator
def test_generate_from_str_semantics(llama3_tok):
    tok = llama3_tok
    cfg = tiny_config(vocab_size=len(tok), num_hidden_layers=2, bos_token_id=tok.bos_id, eos_token_id=tok.eos_id)
    model, *_ = build(cfg, seed=9)
    gen = LLaMA(None, model, tok)
    prompts = ["The quick brown", "hello"]
    outs = gen.generate_from_str(prompts, max_gen_len=6, temperature=0.0)
    assert len(outs) == 2
    for p, o in zip(prompts, outs):
        # decoded from the first BOS, so it includes BOS (tiktoken renders it) and the prompt
        # (generation.py:71-79)
        assert o.startswith("<|begin_of_text|>" + p)
    # token-level: left padding with eos, mask = tokens != eos
    toks = [tok.encode(p, bos=True, eos=False) for p in prompts]
    s = max(map(len, toks))
    t = torch.full((2, s), tok.eos_id, dtype=torch.int32)
    for i, x in enumerate(toks):
        t[i, s - len(x):] = torch.tensor(x)
    seq = gen.generate(t, (t != tok.eos_id).int(), max_gen_len=6, temperature=0.0)
    assert seq.shape == (2, s + 6)
    assert torch.equal(seq[:, :s].int(), t)


def test_example_cli_end_to_end(tmp_path, llama3_tok):
    """examples/generate.py main(): Meta checkpoint + tokenizer -> completions (CPU path)."""
    import importlib.util
    tok_path = str(tmp_path / "tokenizer.model")
    save_tiktoken_bpe(llama3_tok.model.mergeable_ranks, tok_path)
    cfg = tiny_config(vocab_size=len(llama3_tok), num_hidden_layers=2)
    sd = random_meta_state_dict(cfg, seed=4)
    save_meta_checkpoint(sd, params_json_for(cfg, multiple_of=32), str(tmp_path / "ckpt"), n_shards=2,
                         vocab_parallel_embedding=True)
    spec = importlib.util.spec_from_file_location("gen_example", os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "generate.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    outs = mod.main(str(tmp_path / "ckpt"), tok_path, True, max_gen_len=4, temperature=0.0)
    assert len(outs) == 2 and outs[0].startswith("<|begin_of_text|>" + mod.PROMPTS[0])
