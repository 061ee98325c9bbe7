"""Drop-in for the log-probability utilities + welfare of the reference's evaluator.

``StatementEvaluator(evaluation_model, ...).evaluate_statement(statement, issue,
agent_opinions) -> dict`` (src/evaluation.py:50-634) with the same result keys for
the log-probability block (src/evaluation.py:177-394):

  avg_logprob_<agent> / utility_avg_logprob_<agent>   mean token log-prob      (:203-229)
  perplexity_<agent>                                  exp(-avg_logprob)        (:329-335)
  egalitarian / utilitarian / log_nash _welfare_avg_prob and utility_*_logprob
                                                      min / sum / sum log(max(u, 1e-9))
                                                      over avg_prob = mean exp(lp)  (:337-364)
  egalitarian / utilitarian / log_nash _welfare_perplexity
                                                      max / sum / sum log(1/max(ppl, 1e-9))
                                                                                (:367-394)

All agents of all statements are scored in ONE batched pass (per-agent prefix K/V,
cs_logsoftmax_gather, cs_segment_reduce for mean log-prob AND mean prob in one
fold) and every welfare is a cs_welfare_reduce launch over [agents, statements].

Embedding cosine similarity, LLM-as-judge and comparative ranking are remote-API
metrics outside this build: their keys are present and NaN/None,
exactly as the reference reports them when those services are unavailable.
"""
from __future__ import annotations

import math
import time
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from . import ops, runtime, utils
from .methods.prompts import EVAL_SYSTEM

EPS = 1e-9


class StatementEvaluator:
    def __init__(self, evaluation_model: str, llm_judge_model: Optional[str] = None,
                 openai_client: Optional[Any] = None, include_llm_judge: bool = False,
                 include_comparative_ranking: bool = True,
                 embedding_model: str = "BAAI/bge-large-en-v1.5", verbose: bool = True):
        self.evaluation_model = evaluation_model
        self.embedding_model = embedding_model
        self.verbose = verbose
        self.llm_judge_model = llm_judge_model
        self.openai_client = openai_client
        # remote-only metrics: disabled, as the reference does without an OpenAI client
        self.include_llm_judge = False
        self.include_comparative_ranking = False
        self._judge_requested = include_llm_judge

    # --- batched core ---------------------------------------------------------------
    @runtime.serialized("evaluation_model")
    def agent_utilities(self, statements: List[str], issue: str, agent_opinions: Dict[str, str]):
        """Per (agent, statement): mean log-prob and mean prob, as [A, S] device tensors."""
        engine, tok = runtime.get_engine(self.evaluation_model)
        prefixes = [tok.chat_prefix(EVAL_SYSTEM.format(issue=issue, opinion=op), "")
                    for op in agent_opinions.values()]
        cache = engine.prefill(prefixes)
        A, S = len(prefixes), len(statements)
        ids = [tok.encode(s) for s in statements]
        owner = [a for a in range(A) for _ in range(S)]
        conts = [ids[s] for _ in range(A) for s in range(S)]
        lp = engine.score(cache, owner, conts)
        seg = ops.segment_reduce(lp, engine.offsets(conts, engine.device))
        cnt = seg["count"].to(torch.float32).view(A, S)
        nan = torch.full_like(cnt, float("nan"))
        avg_lp = torch.where(cnt > 0, seg["sum_lp"].view(A, S) / cnt.clamp(min=1), nan)
        avg_p = torch.where(cnt > 0, seg["sum_p"].view(A, S) / cnt.clamp(min=1), nan)
        # pairs whose user prompt the reference's find() locates elsewhere: text-compat path
        for a, op in enumerate(agent_opinions.values()):
            system = EVAL_SYSTEM.format(issue=issue, opinion=op)
            for si, st in enumerate(statements):
                where = utils.span_check(tok, system, st)
                if where == utils.SPAN_NONE:      # the reference's call returns ([], [])
                    avg_lp[a, si] = float("nan")
                    avg_p[a, si] = float("nan")
                elif where == utils.SPAN_ELSEWHERE:
                    m_lp, m_p, _ = utils.text_compat_mean(self.evaluation_model, system, st)
                    avg_lp[a, si] = m_lp
                    avg_p[a, si] = m_p
        return avg_lp.contiguous(), avg_p.contiguous()

    def evaluate_statements_batched(self, statements: List[str], issue: str,
                                    agent_opinions: Dict[str, str]) -> List[Dict[str, Any]]:
        t0 = time.time()
        agents = list(agent_opinions)
        avg_lp, avg_p = self.agent_utilities(statements, issue, agent_opinions)
        w = {
            "egalitarian_welfare_avg_prob": ops.welfare(avg_p, "min"),
            "utilitarian_welfare_avg_prob": ops.welfare(avg_p, "sum"),
            "log_nash_welfare_avg_prob": ops.welfare(avg_p, "sumlog", eps=EPS),
        }
        w = {k: v.double().cpu().numpy() for k, v in w.items()}
        lp_h = avg_lp.double().cpu().numpy()
        # perplexity welfare in float64 on the host, exactly as src/evaluation.py:329-381
        # (np.exp of the float64 log-prob: an average below -88.7 is a finite float64
        # perplexity that an fp32 exp would turn into inf and drop from the fold)
        with np.errstate(over="ignore"):
            ppl_h = np.exp(-lp_h)
        for kind in ("egalitarian", "utilitarian", "log_nash"):
            w[f"{kind}_welfare_perplexity"] = np.full(len(statements), np.nan)
        for s in range(len(statements)):
            pp = [ppl_h[a, s] for a in range(lp_h.shape[0]) if np.isfinite(lp_h[a, s])]
            if pp:
                w["egalitarian_welfare_perplexity"][s] = max(pp)
                w["utilitarian_welfare_perplexity"][s] = sum(pp)
                w["log_nash_welfare_perplexity"][s] = sum(np.log([1.0 / max(x, EPS) for x in pp]))
        out = []
        for s in range(len(statements)):
            r: Dict[str, Any] = {"statement_embedding": None}
            for a, aid in enumerate(agents):
                v = lp_h[a, s]
                r[f"avg_logprob_{aid}"] = None if math.isnan(v) else float(v)
                r[f"utility_avg_logprob_{aid}"] = r[f"avg_logprob_{aid}"]
                r[f"cosine_similarity_{aid}"] = None
                r[f"utility_cosine_similarity_{aid}"] = None
            for kind in ("egalitarian", "utilitarian", "log_nash"):
                r[f"{kind}_welfare_cosine"] = np.nan
                r[f"utility_{kind}_welfare_cosine"] = np.nan
            for a, aid in enumerate(agents):
                if not math.isnan(lp_h[a, s]) and math.isfinite(lp_h[a, s]):
                    r[f"perplexity_{aid}"] = float(ppl_h[a, s])
            for kind in ("egalitarian", "utilitarian", "log_nash"):
                val = float(w[f"{kind}_welfare_avg_prob"][s])
                r[f"{kind}_welfare_avg_prob"] = val
                r[f"utility_{kind}_welfare_logprob"] = val
            for kind in ("egalitarian", "utilitarian", "log_nash"):
                r[f"{kind}_welfare_perplexity"] = float(w[f"{kind}_welfare_perplexity"][s])
            if self._judge_requested:
                for key in ("egalitarian_welfare_llm_judge", "utilitarian_welfare_llm_judge",
                            "log_nash_welfare_llm_judge", "llm_judge_egalitarian_welfare",
                            "llm_judge_utilitarian_welfare", "llm_judge_log_nash_welfare"):
                    r[key] = np.nan
            r["evaluation_time_s"] = (time.time() - t0) / max(1, len(statements))
            out.append(r)
        return out

    # --- reference entry points -----------------------------------------------------
    def evaluate_statements(self, statements: Dict[str, Any], issue: str,
                            agent_opinions: Dict[str, str]):
        """DataFrame of evaluation rows (src/evaluation.py:895-1019 contract), all statements
        scored in one batched pass.  Row layout: method, issue, statement,
        method_with_params, [param_*], [seed], [original_row_index], evaluation_time_s, then
        the evaluate_statement keys without the embedding."""
        import pandas as pd

        keys = list(statements)
        texts, seeds, idxs = [], [], []
        for k in keys:
            d = statements[k]
            if isinstance(d, dict):
                texts.append(d.get("statement", ""))
                seeds.append(d.get("seed"))
                idxs.append(d.get("row_index"))
            else:
                texts.append(d)
                seeds.append(None)
                idxs.append(None)
        results = self.evaluate_statements_batched(texts, issue, agent_opinions) if keys else []
        rows = []
        for k, text, seed, ridx, res in zip(keys, texts, seeds, idxs, results):
            base, params, seed_from_key = _parse_method_key(k)
            row = {"method": base, "issue": issue, "statement": text, "method_with_params": k}
            row.update(params)
            final_seed = seed if seed is not None else seed_from_key
            if final_seed is not None:
                row["seed"] = final_seed
            if ridx is not None:
                row["original_row_index"] = ridx
            row["evaluation_time_s"] = res.pop("evaluation_time_s", 0.0)
            for kk, v in res.items():
                if kk != "statement_embedding":
                    row[kk] = v
            rows.append(row)
        return pd.DataFrame(rows)

    def evaluate_results_file(self, results_path, config_path=None, output_dir=None,
                              is_seed_specific: bool = False):
        """Evaluate every statement of a results.csv and write evaluation_results.csv +
        evaluation_config.yaml in the reference's layout (src/evaluation.py:1072-1428),
        which improved_aggregation.py consumes unchanged.  Returns the merged rows."""
        from pathlib import Path

        import pandas as pd
        import yaml

        results_path = Path(results_path)
        results_dir = results_path.parent
        config_path = Path(config_path) if config_path else results_dir / "config.yaml"
        if not results_path.exists():
            raise FileNotFoundError(f"Results file not found: {results_path}")
        df = pd.read_csv(results_path)
        statements = {}
        for _, row in df.iterrows():
            method = row.get("method", "Unknown method")
            stmt = row.get("statement", "No statement generated")
            if stmt == "ERROR" or pd.isna(stmt):
                continue
            params = {c: row[c] for c in row.index if c.startswith("param_") and pd.notna(row[c])}
            seed = row["seed"] if "seed" in row and pd.notna(row["seed"]) else None
            key = utils.create_method_identifier(method, params, include_seed=seed is not None,
                                                 seed_value=seed)
            statements[key] = {"statement": stmt, "seed": seed, "row_index": row.name}
        cfg = yaml.safe_load(open(config_path)) if config_path.exists() else None
        issue = (cfg or {}).get("scenario", {}).get("issue")
        opinions = (cfg or {}).get("scenario", {}).get("agent_opinions", {})
        if not issue or not opinions:
            raise ValueError("Could not extract issue and agent opinions from config. "
                             "Please provide a valid config file.")
        if output_dir is None:
            name = self.evaluation_model.replace("/", "_")
            output_dir = results_dir / f"posthoc_eval_{name}_judge_no_judge"
        output_dir = Path(output_dir)
        out_dir = output_dir if is_seed_specific else output_dir / "seed_0"
        out_dir.mkdir(parents=True, exist_ok=True)
        ev = self.evaluate_statements(statements, issue, opinions)
        ev.to_csv(out_dir / "evaluation_results.csv", index=False)
        with open(out_dir / "evaluation_config.yaml", "w") as f:
            yaml.dump({"original_config": cfg, "evaluation": {
                "evaluation_model": self.evaluation_model, "embedding_model": self.embedding_model,
                "include_llm_judge": False, "llm_judge_model": None,
                "original_results_path": str(results_path), "statements_evaluated": len(statements),
                "rows_processed": len(ev), "total_rows": len(df)}}, f, default_flow_style=False)
        combined = df.copy()
        by_idx = {r["original_row_index"]: r for _, r in ev.iterrows()} \
            if "original_row_index" in ev.columns else {}
        for i in combined.index:
            if i in by_idx:
                combined.at[i, "evaluation_status"] = "completed"
                for col, v in by_idx[i].items():
                    if col not in ("method", "statement", "issue", "original_row_index") \
                            and col not in df.columns:
                        combined.at[i, col] = v
            else:
                combined.at[i, "evaluation_status"] = "skipped"
        return combined

    def evaluate_statement(self, statement: str, issue: str,
                           agent_opinions: Dict[str, str]) -> Dict[str, Any]:
        r = self.evaluate_statements_batched([statement], issue, agent_opinions)[0]
        r.pop("evaluation_time_s", None)
        return r


def _parse_method_key(key: str):
    """'base (k=v, ...) [seed=s]' -> (base, {param_k: v}, seed) with the reference's parsing
    (src/evaluation.py:938-976): params only when the key ends with ')'."""
    base, params, seed = key, {}, None
    if " (" in key:
        parts = key.split(" (", 1)
        base = parts[0]
        if parts[1].endswith(")"):
            for item in parts[1].rstrip(")").split(", "):
                if "=" in item:
                    name, val = item.split("=", 1)
                    try:
                        val = float(val)
                        if val.is_integer():
                            val = int(val)
                    except ValueError:
                        pass
                    params[f"param_{name}"] = val
    if "[seed=" in key and "]" in key:
        try:
            seed = int(key.split("[seed=", 1)[1].split("]", 1)[0])
        except (ValueError, IndexError):
            pass
    return base, params, seed


def write_results_csv(rows, out_path):
    """results.csv with the reference's column order (src/experiment.py:339-373):
    method, statement, error_message, seed, utility_*, param_*, issue, config_file, rest."""
    import pandas as pd

    df = pd.DataFrame(rows)
    core = ["method", "statement", "error_message", "seed"]
    util = sorted(c for c in df.columns if c.startswith("utility_"))
    par = sorted(c for c in df.columns if c.startswith("param_"))
    other = sorted(c for c in df.columns if c not in core + util + par + ["issue", "config_file"])
    order = [c for c in core + util + par + ["issue", "config_file"] + other if c in df.columns]
    df = df[order]
    df.to_csv(out_path, index=False)
    return df


def evaluate_statement(statement: str, issue: str, agent_opinions: dict,
                       evaluation_model: str) -> dict:
    """Legacy module-level entry point (src/evaluation.py:1433-1470)."""
    return StatementEvaluator(evaluation_model, include_comparative_ranking=False,
                              verbose=False).evaluate_statement(statement, issue, agent_opinions)
