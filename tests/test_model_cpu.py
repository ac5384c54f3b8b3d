"""CPU-side checks of the host mirror: config/state_dict surface, expected-size polynomial,
C-ABI library load + exports (no compute calls without a GPU)."""

import copy
import ctypes
import math

import pytest
import torch

from dphubert_amd.synthetic import HUBERT_BASE_CONFIG, HUBERT_LARGE_CONFIG, WAVLM_BASE_CONFIG
from dphubert_amd.wav2vec2.model import wav2vec2_model
from dphubert_amd.wav2vec2.components import _PolyCtx
from helpers import load_golden, seeded_sd
from oracle import hubert_ref as ref

ALL_UNITS = dict(extractor_prune_conv_channels=True, encoder_prune_attention_heads=True,
                 encoder_prune_attention_layer=True, encoder_prune_feed_forward_intermediate=True,
                 encoder_prune_feed_forward_layer=True)


@pytest.mark.parametrize("cfg", [HUBERT_BASE_CONFIG, HUBERT_LARGE_CONFIG, dict(HUBERT_BASE_CONFIG, **ALL_UNITS),
                                 WAVLM_BASE_CONFIG, dict(WAVLM_BASE_CONFIG, **ALL_UNITS)])
def test_state_dict_schema_matches_reference(cfg):
    m = wav2vec2_model(**copy.deepcopy(cfg))
    ours = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    assert ours == ref.state_dict_shapes(cfg)


def test_base_param_count():
    m = wav2vec2_model(**copy.deepcopy(HUBERT_BASE_CONFIG))
    assert sum(p.numel() for p in m.parameters()) == 94371456   # SURVEY 8(a) a11, measured on the reference


def _eval_poly(model, sd):
    poly, mods = model._num_params_poly()
    name_of = {id(mod): n for n, mod in model.named_modules()}
    l0 = [ref.hc_l0_norm(sd[name_of[id(m)] + ".log_alpha"]).item() for m in mods]
    tot = 0.0
    for k, c in poly.t.items():
        v = c
        for i in k:
            v *= l0[i]
        tot += v
    return tot


@pytest.mark.parametrize("units", [ALL_UNITS, dict(extractor_prune_conv_channels=True,
                                                   encoder_prune_attention_heads=True,
                                                   encoder_prune_feed_forward_intermediate=True), {}])
def test_expected_params_polynomial(units):
    cfg = dict(HUBERT_BASE_CONFIG, encoder_num_layers=3, encoder_use_attention=[True] * 3,
               encoder_use_feed_forward=[True] * 3, encoder_num_heads=[12] * 3,
               encoder_ff_interm_features=[3072] * 3, **units)
    sd = seeded_sd(cfg, 3)
    m = wav2vec2_model(**copy.deepcopy(cfg))
    m.load_state_dict(sd)
    want = float(ref.get_num_params(sd, cfg))
    got = _eval_poly(m, sd)
    assert abs(got - want) <= 1e-6 * want


def test_wavlm_expected_params_and_schema_vs_reference():
    """WavLM: the state_dict schema and the initial expected #params of the reference's own model (fixture g8:
    the relative-position embedding and gate are not counted, as WavLMSelfAttention inherits get_num_params)."""
    fx = load_golden("g8_wavlm.pt")
    cfg = dict(fx["scfg"])
    m = wav2vec2_model(**copy.deepcopy(cfg))
    assert [(k, tuple(v.shape)) for k, v in m.state_dict().items()] == [(k, tuple(s)) for k, s in fx["sd_schema"]]
    sd = seeded_sd(cfg, 0)
    m.load_state_dict(sd)
    assert abs(_eval_poly(m, sd) - fx["num_params_init"]) <= 1e-6 * fx["num_params_init"]


def test_expected_params_matches_golden():
    d = load_golden("g1_ops.pt")["num_params"]
    m = wav2vec2_model(**copy.deepcopy(d["cfg"]))
    sd = seeded_sd(d["cfg"], d["seed"])
    m.load_state_dict(sd)
    assert abs(_eval_poly(m, sd) - float(d["value"])) <= 1e-6 * float(d["value"])


def test_library_loads_and_exports_every_symbol():
    from dphubert_amd import _lib
    L = _lib.lib()
    assert L.missing_symbols == []
    assert L.dph_abi_version() == _lib.ABI_VERSION
    # every symbol declared in include/dphubert_hip.h is exported
    import re
    from pathlib import Path
    hdr = (Path(__file__).resolve().parents[1] / "include" / "dphubert_hip.h").read_text()
    declared = set(re.findall(r"^\s*(?:const char\*|int|int64_t)\s+(dph_\w+)\s*\(", hdr, re.M))
    assert declared, "no declarations parsed"
    for name in declared:
        assert hasattr(L, name), name
    assert declared <= set(_lib.exported_symbols())


def test_abi_rejects_bad_args_without_gpu():
    # argument validation happens on the host before any launch
    from dphubert_amd import _lib
    L = _lib.lib()
    rc = L.dph_layernorm_fwd(None, None, None, None, None, None, None, 0, 768, 1e-5, 0.0, 0, None)
    assert rc == -1
    assert b"null pointer" in L.dph_last_error()


def test_no_cpu_fallback():
    m = wav2vec2_model(**copy.deepcopy(HUBERT_BASE_CONFIG))
    with pytest.raises(ValueError):
        m.extract_features(torch.zeros(2, 16000))     # CPU tensors are rejected, never computed on the host


def test_trace_ranges_name_each_abi_call():
    """DPH_TRACE / _lib.set_trace: every C-ABI call runs inside a torch.profiler.record_function range named after
    its entry point (SURVEY 5 tracing); off by default.  Host-only entry points, so no GPU is needed."""
    from torch.profiler import ProfilerActivity, profile
    from dphubert_amd import _lib
    prev = _lib.set_trace(True)
    det = _lib.deterministic()
    try:
        with profile(activities=[ProfilerActivity.CPU]) as prof:
            _lib.call("dph_set_deterministic", 1)
            _lib.call("dph_defer_reductions", 0)
    finally:
        _lib.set_trace(prev)
        _lib.set_deterministic(det)
    names = {e.name for e in prof.events()}
    assert {"dph::dph_set_deterministic", "dph::dph_defer_reductions"} <= names, sorted(names)[:20]
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        _lib.call("dph_defer_reductions", 0)
    assert not any(e.name.startswith("dph::") for e in prof.events())


def test_discard_reductions_host_only():
    """dph_discard_reductions (ABI 23) empties the deferred-reduction queue without launching anything."""
    from dphubert_amd import _lib
    L = _lib.lib()
    assert L.dph_deferred_reductions() == 0
    assert L.dph_discard_reductions() == 0
    assert L.dph_reductions_pushed() >= 0
