"""Prompt texts and token constants of the reference methods.

These strings are DATA the drop-in must reproduce byte for byte: utilities are
log-probabilities under exactly these prompts.  Each table cites its source
(relative to the reference root).
"""

_REF_SYS = (
    "You are generating a consensus statement that represents the views of multiple participants.\n"
    "Your task is to continue the statement in a way that addresses the issue and considers all "
    "participants' opinions. Be concise and keep the statement short (less than 50 tokens) and "
    "focused. ONLY WRITE THE STATEMENT AND NOTHING ELSE.")
_AGENT_SYS = (
    "You are generating a statement that represents the views of a single participant.\n"
    "Your task is to continue the statement in a way that addresses the issue and considers ONLY "
    "this participant's opinion. Be concise and keep the statement short (less than 50 tokens) "
    "and focused. ONLY WRITE THE STATEMENT AND NOTHING ELSE.")

# src/methods/beam_search.py:26-79
BEAM = dict(
    eos_tokens=frozenset({"<|eot_id|>", "<|end_of_text|>", ".\n\n", ".\n", "\n\n", '."\n\n',
                          "<end_of_turn>", "<eos>"}),
    bias_against=["...", '"', "***", "**", "\n\n\n", "\n\n\n\n", ":", " ...", " .", " •",
                  "<end_of_turn>", "<eos>", "<start_of_turn>"],
    bias_value=-1000000,
    ref_system=_REF_SYS,
    agent_system=_AGENT_SYS,
    ref_user="Issue:\n{issue}\n\nParticipants' opinions:\n{opinions_text}\n\n"
             "Consensus statement (less than 50 tokens):\n",
    agent_user="Issue:\n{issue}\n\nParticipant's opinion:\n{opinion}\n\n"
               "Statement reflecting ONLY this participant's opinion (less than 50 tokens):\n",
)

# src/methods/best_of_n.py:22-35
BON = dict(
    default_reward=-10.0, clip_min=-20.0, clip_max=20.0, eps=1e-9,
    eos_tokens=frozenset({"<|eot_id|>", "<|end_of_text|>"}),
    ref_system=_REF_SYS,
    agent_system=_AGENT_SYS,
    agent_user="Issue: {issue}\n\nAgent's opinion:\n{opinion}\n\n"
               "Statement reflecting this opinion (less than 50 tokens): ",
    ref_user="Issue: {issue}\n\nParticipants' opinions:\n{opinions_text}\n\n"
             "Consensus statement (less than 50 tokens): ",
    # src/methods/best_of_n.py:217-224
    clean_prefixes=["Consensus statement:", "Statement:", "Here is the consensus statement:",
                    "Here is a statement reflecting this opinion:", "Okay, here is the statement:"],
)

# src/methods/finite_lookahead.py:21-33, 317-331, 350
FL = dict(
    default_reward=-10.0, clip_min=-20.0, clip_max=20.0, eps=1e-9,
    ref_system=_REF_SYS,
    agent_system=_AGENT_SYS,
    agent_user="Issue:\n{issue}\n\nAgent's opinion:\n{opinion}\n\n"
               "Statement reflecting this opinion (less than 50 tokens):\n",
    ref_user="Issue:\n{issue}\n\nParticipants' opinions:\n{opinions_text}\n\n"
             "Consensus statement (less than 50 tokens):\n",
    bias_against=["...", '"', "***", "**", "\n\n\n", "\n\n\n\n", ":", " ...", " .", " •",
                  "<end_of_turn>", "<eos>", "<start_of_turn>"],
    bias_value=-1000000,           # generate_text default (src/utils.py:85)
    terminal_tokens=["\n", "\n\n", ".\n\n", '."\n\n'],
    stop_tokens=["\n", "\n\n", ".\n\n"],   # finite_lookahead.py:141-144
)

# src/methods/mcts.py:62-91 (its own, shorter system texts and EOS set)
MCTS = dict(
    eos_tokens=frozenset({"<|eot_id|>", "<|end_of_text|>", ".\n\n", ".\n", "\n\n", '."\n\n'}),
    ref_system=("You are generating a consensus statement that represents the views of multiple "
                "participants.\nYour task is to continue the statement in a way that addresses the "
                "issue and considers all participants' opinions. Be concise and coherent. ONLY WRITE "
                "THE CONSENSUS STATEMENT AND NOTHING ELSE."),
    agent_system=("You are generating a statement that represents the views of a single "
                  "participant.\nYour task is to continue the statement in a way that addresses "
                  "the issue and considers ONLY this participant's opinion. Be concise and "
                  "coherent. ONLY WRITE THE CONSENSUS STATEMENT AND NOTHING ELSE."),
    ref_user="Issue:\n{issue}\n\nParticipants' opinions:\n{opinions_text}\n\nConsensus statement:\n",
    agent_user="Issue:\n{issue}\n\nParticipant's opinion:\n{opinion}\n\n"
               "Statement reflecting ONLY this participant's opinion:\n",
    failure_reward=-100.0,     # mcts.py:497, 566, 650 (failed evaluation / empty rollout)
)

# src/evaluation.py:182-186
EVAL_SYSTEM = ("Issue: {issue}. Agent's Opinion: {opinion}. Here is a consensus statement that "
               "perfectly aligns with the agent's opinion:")


def opinions_text(agent_opinions: dict) -> str:
    """'Participant i: ...' blocks joined by blank lines (beam_search.py:139-144)."""
    return "\n\n".join(f"Participant {i + 1}: {op}" for i, op in enumerate(agent_opinions.values()))
