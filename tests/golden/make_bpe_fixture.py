"""Build the byte-level BPE tokenizer fixture (tests/golden/bpe_fixture/).

No pretrained tokenizer is available offline, so the real-model path's
tokenizer.json loader, its chat templates and the benchmarks' prompt lengths are pinned
on a tokenizer trained HERE, in Hugging Face `tokenizers` format, on the reference's own
text data (scenario texts of configs/**/*.yaml and the published statements of
results/**/results.csv): a Llama-3-style byte-level BPE (same pre-tokenizer regex,
ByteLevel decoder) with the Llama-3 and Gemma-2 special tokens, vocabulary 8192 — English
scenario text compresses to ~4 characters per token, as the real tokenizers do, so
prompt token counts are realistic.

Outputs (committed; the reference never travels to the GPU box):
  tokenizer.json          the tokenizer
  tokenizer_config.json   bos / eos and the Llama-3 chat template (jinja), the one
                          transformers' apply_chat_template renders
Run from the repo root:  python tests/golden/make_bpe_fixture.py [/root/reference]
"""
import csv
import glob
import json
import os
import sys

from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers, trainers

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "bpe_fixture")
SPECIALS = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>", "<|end_header_id|>",
            "<|eot_id|>", "<bos>", "<eos>", "<start_of_turn>", "<end_of_turn>", "<pad>"]
# the Llama-3 pre-tokenizer split pattern (public tokenizer.json of Meta-Llama-3)
LLAMA3_SPLIT = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?"
                r"[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")
# Meta-Llama-3-8B-Instruct's chat template (tokenizer_config.json)
LLAMA3_TEMPLATE = (
    "{% set loop_messages = messages %}{% for message in loop_messages %}"
    "{% set content = '<|start_header_id|>' + message['role'] + '<|end_header_id|>\n\n'"
    "+ message['content'] | trim + '<|eot_id|>' %}{% if loop.index0 == 0 %}"
    "{% set content = bos_token + content %}{% endif %}{{ content }}{% endfor %}"
    "{% if add_generation_prompt %}{{ '<|start_header_id|>assistant<|end_header_id|>\n\n' }}"
    "{% endif %}")


def corpus(ref_root):
    texts = []
    for f in sorted(glob.glob(os.path.join(ref_root, "configs", "**", "*.yaml"), recursive=True)):
        texts.append(open(f, encoding="utf-8").read())
    csv.field_size_limit(1 << 30)
    for f in sorted(glob.glob(os.path.join(ref_root, "results", "**", "results.csv"), recursive=True)):
        with open(f, encoding="utf-8") as fh:
            for row in csv.DictReader(fh):
                for k in ("statement", "pre_brushup_statement"):
                    if row.get(k):
                        texts.append(row[k])
    return texts


def build(ref_root="/root/reference"):
    tk = Tokenizer(models.BPE())
    tk.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(LLAMA3_SPLIT), behavior="isolated"),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    tk.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=8192, min_frequency=2, special_tokens=SPECIALS,
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                                  show_progress=False)
    tk.train_from_iterator(corpus(ref_root), trainer=trainer)
    os.makedirs(OUT, exist_ok=True)
    tk.save(os.path.join(OUT, "tokenizer.json"))
    with open(os.path.join(OUT, "tokenizer_config.json"), "w") as f:
        json.dump({"bos_token": "<|begin_of_text|>", "eos_token": "<|eot_id|>",
                   "chat_template": LLAMA3_TEMPLATE, "model_max_length": 131072,
                   "tokenizer_class": "PreTrainedTokenizerFast"}, f, indent=1)
    return tk


if __name__ == "__main__":
    t = build(sys.argv[1] if len(sys.argv) > 1 else "/root/reference")
    print("vocab", t.get_vocab_size(), "->", OUT)
