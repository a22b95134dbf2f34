"""Synthetic interpreter states for config 5: text_adventure.json5 forked states.

Configs 2-4 are generated in HBM by the library itself (ie_synth_*, ie_common.h). Config 5 is a
batch over many *states*: each state is an inserts dict at the top of the game loop
(examples/text_adventure.json5:26, label '@loop') — the program's default inserts (:4-15) plus
the keys the loop reads: scenario, stage, history_list (2-36 tagged entries), the joined
history texts (0.2-8 KB), output, new_user_input. The batch resolves the per-iteration call
stream (recorded from the reference, tests/golden/config5_stream.json) against every state, one
table per state (a table set, ie_table_set_build).

Deterministic: splitmix64 seeded per state, so the bench and the tests build identical states.
"""

_WORDS = ("the knight walks into a dark hall and sees a door to the north there is a faint light "
          "you hear steps behind you a guard asks for your name the road is long and cold "
          "an old woman sells bread at the gate ask about the castle open the chest look around "
          "take the sword go north talk to the guard the wizard smiles and nods é € 😀").split()
_TAGS = (("<action>", "</action>"), ("<action-output>", "</action-output>"), ("<query>", "</query>"),
         ("<query-output>", "</query-output>"), ("<first-output>", "</first-output>"))
STAGES = ("first", "action", "query", "undo")


def _splitmix(s):
    s = (s + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = s
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return s, z ^ (z >> 31)


class _Rng:
    def __init__(self, seed):
        self.s = seed & 0xFFFFFFFFFFFFFFFF

    def next(self):
        self.s, z = _splitmix(self.s)
        return z

    def below(self, n):
        return self.next() % n

    def words(self, lo, hi):
        return " ".join(_WORDS[self.below(len(_WORDS))] for _ in range(lo + self.below(hi - lo + 1)))


def history_entry(rng, k):
    """One tagged history entry as the program appends them (text_adventure.json5:215-258)."""
    if k == 0:
        o, c = _TAGS[4]
        return o + rng.words(20, 60) + c
    if k % 2 == 1:
        o, c = _TAGS[0] if rng.below(4) else _TAGS[2]
        return o + rng.words(2, 10) + c
    o, c = _TAGS[1] if rng.below(4) else _TAGS[3]
    return o + rng.words(15, 55) + c


def _strip_tags(text):
    # the effect of the program's markup replace_map (text_adventure.json5:33-49) on generated text
    for o, c in _TAGS:
        text = text.replace(o, "").replace(c, "")
    return text


def state_inserts(defaults, index, seed=0x1E5EED05, max_entries=36):
    """The inserts of synthetic state `index` at label '@loop' plus the keys the loop sets before
    its first chat. `defaults` are the program's default inserts (from the recorded stream)."""
    rng = _Rng(seed ^ (index * 0xD1B54A32D192ED03))
    n = 2 + rng.below(max_entries - 1)
    hist = [history_entry(rng, k) for k in range(n)]
    base = "\n\n".join(hist)
    ins = dict(defaults)
    ins["scenario"] = "This is a text adventure game where you play as " + rng.words(4, 16) + "."
    ins["stage"] = STAGES[rng.below(3)]  # 'undo' loops once more before a chat: the stream covers it
    ins["history_list"] = hist
    ins["history_text_base"] = base
    ins["history_text_printed"] = _strip_tags(base)
    ins["history_text_llm"] = base.replace("  ", " ")
    ins["output"] = "(unset)"
    ins["new_user_input"] = rng.words(2, 8)
    ins["maybe_input"] = ins["new_user_input"]
    # what the loop's math commands compute from the history (text_adventure.json5:264-302)
    lo, hi = int(ins.get("min_history_turns", 4)), int(ins.get("max_history_turns", 18))
    ins["isodd"] = n % 2
    ins["length_history"] = n
    ins["n_summarize"] = n - 2 * lo
    ins["should_summarize"] = (n > 2 * hi) - (n < 2 * hi)
    ins["summarize_ok"] = (n > 2 * lo) - (n < 2 * lo)
    return ins
