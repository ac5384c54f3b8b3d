"""Algorithmic work of one distill step: the FLOPs the MFMA roofline is priced on and the bytes of the
HBM-bound kernels.  Used by bench.py (roofline, TFLOP/s) and by the training log (``mfma_util`` / ``hbm_gbps`` next to
the reference's lightning.py:277-295 keys, SURVEY 2 "Metrics / logging")."""

MFMA_PEAK_TFLOPS = 2500.0        # MI355X dense bf16 (MI355X_MICROARCH.md)
HBM_PEAK_GBPS = 8000.0           # MI355X HBM3E


def conv_frames(cfg: dict, samples: int) -> int:
    L = samples
    for _, k, s_ in cfg["extractor_conv_layer_config"]:
        L = (L - k) // s_ + 1
    return L


def forward_flops(cfg: dict, samples: int) -> float:
    """Dense forward FLOPs of one utterance through extract_features: conv frontend, feature
    projection, positional conv, per layer q/k/v/out projections, QK^T + PV and the FFN, at the config's (possibly
    pruned, ragged) widths."""
    L, cin, f = samples, 1, 0.0
    for cout, k, s_ in cfg["extractor_conv_layer_config"]:
        L = (L - k) // s_ + 1
        f += 2.0 * cin * cout * k * L
        cin = cout
    T, D = L, cfg["encoder_embed_dim"]
    f += 2.0 * cin * D * T
    f += 2.0 * D * (D // cfg["encoder_pos_conv_groups"]) * cfg["encoder_pos_conv_kernel"] * T
    heads = cfg.get("encoder_num_heads") or [len(h) for h in cfg["encoder_remaining_heads"]]
    hd = cfg.get("encoder_head_dim", 64)
    for l in range(cfg["encoder_num_layers"]):
        if cfg["encoder_use_attention"][l] and heads[l] > 0:
            e = heads[l] * hd
            f += 2.0 * T * D * 3 * e + 2.0 * T * e * D + 4.0 * T * T * e
        if cfg["encoder_use_feed_forward"][l]:
            f += 4.0 * T * D * cfg["encoder_ff_interm_features"][l]
    return f


def step_flops_per_utt(tcfg: dict, scfg: dict, n_distill: int, samples: int) -> float:
    """teacher forward + 3 x (student forward + distill projections) per utterance."""
    T = conv_frames(tcfg, samples)
    proj = n_distill * 2.0 * T * scfg["encoder_embed_dim"] * tcfg["encoder_embed_dim"]
    return forward_flops(tcfg, samples) + 3.0 * (forward_flops(scfg, samples) + proj)


def step_hbm_bytes_per_utt(tcfg: dict, scfg: dict, samples: int) -> float:
    """Algorithmic HBM bytes per utterance of the step's bandwidth-bound kernels (DESIGN 4 "HBM" rows), not counting
    the GEMM / attention operand streams (priced on the MFMA roofline): the LayerNorms (forward reads x and writes y,
    2 + 2 B per element; backward reads dy and x and writes dx, 6 B; two per layer; teacher forward only) and the
    conv0 GroupNorm activation stream (bf16 [L0][C]: written by each forward, read by the student backward)."""
    T = conv_frames(tcfg, samples)
    b = 0.0
    for cfg, train in ((tcfg, False), (scfg, True)):
        D = cfg["encoder_embed_dim"]
        per = 2 * (4 + (6 if train else 0))
        b += cfg["encoder_num_layers"] * per * T * D
        cout, k, s_ = cfg["extractor_conv_layer_config"][0]
        L0 = (samples - k) // s_ + 1
        b += (2 if train else 1) * L0 * cout * 2
    return b


def optimizer_hbm_bytes(trainable_params: int) -> float:
    """AdamW (optim.hip): reads param, grad, exp_avg, exp_avg_sq (16 B), writes param, exp_avg, exp_avg_sq (12 B) and
    the bf16 GEMM image (2 B) per trainable parameter."""
    return 30.0 * trainable_params
