"""Local Hugging Face checkpoints -> ScoringEngine (the real-model path).

The reference names remote models ("meta-llama/Meta-Llama-3.1-8B-Instruct-Turbo",
"google/gemma-2-9b-it") served by the Together API (src/utils.py:69-74).  Here such an id
resolves (runtime.get_engine) to a local checkpoint directory in the published layout:

    config.json               LlamaForCausalLM / Gemma2ForCausalLM hyper-parameters
    *.safetensors             weights under the Hugging Face parameter names
    tokenizer.json            the tokenizer (+ tokenizer_config.json: chat template)

Weights are read with safetensors (no pickle), mapped to the engine's names (the inverse
of model.hf_state_dict) and cast to the engine dtype on the device; the q/k/v and
gate/up projections are then fused per layer as for random-init models.
"""
from __future__ import annotations

import glob
import json
import os
from typing import Dict, Optional, Tuple

import torch

from .engine import ScoringEngine
from .model import Model, ModelConfig
from .tokenizer import BPETokenizer

_FAMILY = {"llama": "llama3", "gemma2": "gemma2"}


def config_from_hf(conf: dict, name: str = "checkpoint") -> ModelConfig:
    """ModelConfig from a Hugging Face config.json (Llama-3.x or Gemma-2)."""
    mt = conf.get("model_type")
    if mt not in _FAMILY:
        raise ValueError(f"unsupported model_type {mt!r} (Llama-3 'llama' or Gemma-2 'gemma2')")
    fam = _FAMILY[mt]
    H = conf["num_attention_heads"]
    d = conf["hidden_size"]
    rs = conf.get("rope_scaling")
    if rs is not None and rs.get("rope_type", rs.get("type")) not in ("llama3",):
        raise ValueError(f"unsupported rope_scaling {rs!r}")
    kw = dict(name=name, family=fam, vocab=conf["vocab_size"], d_model=d,
              n_layers=conf["num_hidden_layers"], n_heads=H,
              n_kv_heads=conf.get("num_key_value_heads", H),
              head_dim=conf.get("head_dim") or d // H, d_ff=conf["intermediate_size"],
              rope_theta=float(conf.get("rope_theta", 10000.0)),
              rms_eps=float(conf.get("rms_norm_eps", 1e-6)),
              tie_embeddings=bool(conf.get("tie_word_embeddings", fam == "gemma2")),
              rope_scaling=({k: rs[k] for k in ("factor", "low_freq_factor", "high_freq_factor",
                                                 "original_max_position_embeddings")}
                            if rs else None))
    if fam == "gemma2":
        kw.update(final_softcap=float(conf.get("final_logit_softcapping") or 0.0),
                  attn_softcap=float(conf.get("attn_logit_softcapping") or 0.0),
                  sliding_window=int(conf.get("sliding_window") or 0),
                  query_pre_attn_scalar=(float(conf["query_pre_attn_scalar"])
                                         if conf.get("query_pre_attn_scalar") else None))
    return ModelConfig(**kw)


def hf_name_map(cfg: ModelConfig) -> Dict[str, str]:
    """Hugging Face parameter name -> engine weight name."""
    m = {"model.embed_tokens.weight": "embed", "model.norm.weight": "norm"}
    if not cfg.tie_embeddings:
        m["lm_head.weight"] = "lm_head"
    for i in range(cfg.n_layers):
        p, q = f"l{i}.", f"model.layers.{i}."
        m.update({q + "self_attn.q_proj.weight": p + "wq", q + "self_attn.k_proj.weight": p + "wk",
                  q + "self_attn.v_proj.weight": p + "wv", q + "self_attn.o_proj.weight": p + "wo",
                  q + "mlp.gate_proj.weight": p + "w_gate", q + "mlp.up_proj.weight": p + "w_up",
                  q + "mlp.down_proj.weight": p + "w_down",
                  q + "input_layernorm.weight": p + "attn_norm"})
        if cfg.family == "gemma2":
            m[q + "post_attention_layernorm.weight"] = p + "post_attn_norm"
            m[q + "pre_feedforward_layernorm.weight"] = p + "mlp_norm"
            m[q + "post_feedforward_layernorm.weight"] = p + "post_mlp_norm"
        else:
            m[q + "post_attention_layernorm.weight"] = p + "mlp_norm"
    return m


def load_weights(path: str, cfg: ModelConfig, device, dtype) -> Dict[str, torch.Tensor]:
    from safetensors import safe_open

    files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
    if not files:
        raise FileNotFoundError(f"no *.safetensors under {path}")
    names = hf_name_map(cfg)
    w: Dict[str, torch.Tensor] = {}
    for f in files:
        with safe_open(f, framework="pt", device="cpu") as sf:
            for k in sf.keys():
                if k in names:
                    w[names[k]] = sf.get_tensor(k).to(device=device, dtype=dtype)
    missing = [n for n in names.values() if n not in w]
    if missing:
        raise ValueError(f"checkpoint {path} lacks weights: {missing[:6]}{' ...' if len(missing) > 6 else ''}")
    return w


def load_model(path: str, device=None, dtype=torch.bfloat16) -> Model:
    with open(os.path.join(path, "config.json")) as f:
        cfg = config_from_hf(json.load(f), name=os.path.basename(os.path.normpath(path)))
    dev = torch.device(device) if device is not None else \
        torch.device("cuda", torch.cuda.current_device())
    return Model(cfg, dev, dtype, weights=load_weights(path, cfg, dev, dtype))


def load_engine(path: str, device=None, dtype=torch.bfloat16,
                **engine_kw) -> Tuple[ScoringEngine, BPETokenizer]:
    """(ScoringEngine, tokenizer) of a local checkpoint directory."""
    model = load_model(path, device, dtype)
    tok = BPETokenizer(path, family=model.cfg.family, vocab_size=model.cfg.vocab)
    return ScoringEngine(model, **engine_kw), tok


def save_checkpoint(model: Model, path: str, tokenizer_dir: Optional[str] = None) -> None:
    """Write ``model`` in the published layout (config.json + model.safetensors, plus the
    tokenizer files of ``tokenizer_dir``): the offline fixtures of the loader's tests."""
    import shutil

    from safetensors.torch import save_file

    from .model import hf_state_dict

    c = model.cfg
    os.makedirs(path, exist_ok=True)
    conf = {"model_type": "llama" if c.family == "llama3" else "gemma2",
            "architectures": ["LlamaForCausalLM" if c.family == "llama3" else "Gemma2ForCausalLM"],
            "vocab_size": c.vocab, "hidden_size": c.d_model, "num_hidden_layers": c.n_layers,
            "num_attention_heads": c.n_heads, "num_key_value_heads": c.n_kv_heads,
            "head_dim": c.head_dim, "intermediate_size": c.d_ff, "rope_theta": c.rope_theta,
            "rms_norm_eps": c.rms_eps, "tie_word_embeddings": c.tie_embeddings,
            "max_position_embeddings": 8192, "torch_dtype": "float32"}
    if c.rope_scaling:
        conf["rope_scaling"] = dict(c.rope_scaling, rope_type="llama3")
    if c.family == "gemma2":
        conf.update(final_logit_softcapping=c.final_softcap, attn_logit_softcapping=c.attn_softcap,
                    sliding_window=c.sliding_window,
                    query_pre_attn_scalar=(int(c.query_pre_attn_scalar)
                                           if float(c.query_pre_attn_scalar).is_integer()
                                           else c.query_pre_attn_scalar),
                    hidden_activation="gelu_pytorch_tanh", hidden_act="gelu_pytorch_tanh")
    else:
        conf.update(hidden_act="silu", attention_bias=False, mlp_bias=False)
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(conf, f, indent=1)
    sd = {k: v.detach().to("cpu").contiguous().clone() for k, v in hf_state_dict(model).items()}
    if c.tie_embeddings:
        sd.pop("lm_head.weight", None)
    save_file(sd, os.path.join(path, "model.safetensors"))
    if tokenizer_dir:
        for n in ("tokenizer.json", "tokenizer_config.json"):
            src = os.path.join(tokenizer_dir, n)
            if os.path.exists(src):
                shutil.copy(src, os.path.join(path, n))
