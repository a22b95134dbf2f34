"""Program loading for the runner side of the hot path: a JSON5 reader, the
reference's `line:` injection, task labelling, and a minimal runner whose only job is the per-task
interpolation pre-pass through the device resolver (config 1: examples/hello_world.json5).

Reference behaviour restated (src/interpolation_engine/interpolation_engine.py, read as text):
  add_line_numbers(text)          py:2267-2276   (rust-project/src/parser.rs:72-92 is the same rule)
  load(path) -> (program, state)  py:2283-2312   (the md5 load cache is a UI nicety, not restated)
  task labels                     py:1042-1072   (validate_program's traceback_label assignment only;
                                                  its static key analysis is out of scope)
  ARGn pre-seeding                py:2343-2349   (the recursive_escape rule on each argument)
  execute_task pre-pass           py:1501        (recursive_interpolate of every task)

The `json5` package the reference imports (py:456, 2300) is not installed here, so `loads` is this
module's own reader of the JSON5 grammar (ECMAScript 5 literals): comments, unquoted identifier
keys, single- or double-quoted strings with every ES5 escape (a backslash before any other
character yields that character, so '\\{' reads as '{'), line continuations, trailing commas, hex,
leading/trailing-dot and signed numbers, Infinity/NaN, duplicate keys last-wins. Integers come
back as int, other numbers as float (what the json5 package returns).
"""
import copy
import math
import re

__all__ = ["loads", "add_line_numbers", "label_tasks", "load_program", "Runner", "JSON5Error"]


class JSON5Error(ValueError):
    pass


_WS = set(" \t\n\r\v\f\u00a0\u1680\u2028\u2029\u202f\u205f\u3000\ufeff" + "".join(chr(c) for c in range(0x2000, 0x200B)))
_ESC = {"b": "\b", "f": "\f", "n": "\n", "r": "\r", "t": "\t", "v": "\v", "'": "'", '"': '"', "\\": "\\"}
_LINE_TERM = "\n\r\u2028\u2029"


class _Reader:
    def __init__(self, text):
        self.s = text
        self.i = 0

    def err(self, msg):
        line = self.s.count("\n", 0, self.i) + 1
        col = self.i - (self.s.rfind("\n", 0, self.i) + 1) + 1
        raise JSON5Error("%s at line %d column %d" % (msg, line, col))

    def skip(self):
        s, n = self.s, len(self.s)
        while self.i < n:
            c = s[self.i]
            if c in _WS:
                self.i += 1
            elif s.startswith("//", self.i):
                while self.i < n and s[self.i] not in _LINE_TERM:
                    self.i += 1
            elif s.startswith("/*", self.i):
                j = s.find("*/", self.i + 2)
                if j < 0:
                    self.err("unterminated comment")
                self.i = j + 2
            else:
                return

    def value(self):
        self.skip()
        if self.i >= len(self.s):
            self.err("unexpected end of input")
        c = self.s[self.i]
        if c == "{":
            return self.obj()
        if c == "[":
            return self.arr()
        if c in "'\"":
            return self.string()
        return self.literal()

    def obj(self):
        self.i += 1
        out = {}
        while True:
            self.skip()
            if self.i >= len(self.s):
                self.err("unterminated object")
            if self.s[self.i] == "}":
                self.i += 1
                return out
            key = self.string() if self.s[self.i] in "'\"" else self.ident()
            self.skip()
            if self.i >= len(self.s) or self.s[self.i] != ":":
                self.err("expected ':'")
            self.i += 1
            out[key] = self.value()
            self.skip()
            if self.i < len(self.s) and self.s[self.i] == ",":
                self.i += 1
            elif self.i < len(self.s) and self.s[self.i] == "}":
                continue
            else:
                self.err("expected ',' or '}'")

    def arr(self):
        self.i += 1
        out = []
        while True:
            self.skip()
            if self.i >= len(self.s):
                self.err("unterminated array")
            if self.s[self.i] == "]":
                self.i += 1
                return out
            out.append(self.value())
            self.skip()
            if self.i < len(self.s) and self.s[self.i] == ",":
                self.i += 1
            elif self.i < len(self.s) and self.s[self.i] == "]":
                continue
            else:
                self.err("expected ',' or ']'")

    def ident(self):
        s, j = self.s, self.i
        out = []
        while j < len(s):
            c = s[j]
            if c == "\\" and s.startswith("\\u", j):
                out.append(chr(int(s[j + 2:j + 6], 16)))
                j += 6
                continue
            if c.isalnum() or c in "_$" or (ord(c) > 127 and (c.isidentifier() or ("a" + c).isidentifier())):
                out.append(c)
                j += 1
                continue
            break
        if j == self.i or out[0].isdigit():
            self.err("expected a key")
        self.i = j
        return "".join(out)

    def string(self):
        s = self.s
        q = s[self.i]
        j = self.i + 1
        out = []
        while True:
            if j >= len(s):
                self.i = j
                self.err("unterminated string")
            c = s[j]
            if c == q:
                self.i = j + 1
                return "".join(out)
            if c in "\n\r":
                self.i = j
                self.err("line break in string")
            if c != "\\":
                out.append(c)
                j += 1
                continue
            e = s[j + 1] if j + 1 < len(s) else ""
            if e in _ESC:
                out.append(_ESC[e])
                j += 2
            elif e == "0" and not (j + 2 < len(s) and s[j + 2].isdigit()):
                out.append("\0")
                j += 2
            elif e == "x":
                out.append(chr(int(s[j + 2:j + 4], 16)))
                j += 4
            elif e == "u":
                cp = int(s[j + 2:j + 6], 16)
                j += 6
                if 0xD800 <= cp < 0xDC00 and s.startswith("\\u", j):
                    lo = int(s[j + 2:j + 6], 16)
                    if 0xDC00 <= lo < 0xE000:
                        cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00)
                        j += 6
                out.append(chr(cp))
            elif e == "\r":  # line continuation
                j += 3 if s.startswith("\r\n", j + 1) else 2
            elif e in "\n\u2028\u2029":
                j += 2
            elif e == "":
                self.i = j
                self.err("unterminated string")
            else:  # NonEscapeCharacter: the character itself
                out.append(e)
                j += 2

    _NUM = re.compile(r"[+-]?(?:0[xX][0-9a-fA-F]+|Infinity|NaN|(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?)")

    def literal(self):
        s = self.s
        for word, val in (("true", True), ("false", False), ("null", None)):
            if s.startswith(word, self.i):
                self.i += len(word)
                return val
        m = self._NUM.match(s, self.i)
        if not m:
            self.err("unexpected character %r" % s[self.i])
        t = m.group(0)
        self.i = m.end()
        sign = -1 if t[0] == "-" else 1
        body = t.lstrip("+-")
        if body == "Infinity":
            return sign * math.inf
        if body == "NaN":
            return math.nan
        if body[:2] in ("0x", "0X"):
            return sign * int(body[2:], 16)
        if re.fullmatch(r"\d+", body):
            return sign * int(body)
        return sign * float(body)


def loads(text):
    """Parse one JSON5 value (the whole text)."""
    r = _Reader(text)
    v = r.value()
    r.skip()
    if r.i != len(text):
        r.err("trailing characters")
    return v


# the reference's `cmd: '...'` matcher (py:2270): the key `cmd` bare or quoted, a quoted value,
# then ',' or '}' — the task gets `, line:N` injected after its value, N = the 1-based line
_CMD = re.compile(r"""(\bcmd\b|"cmd"|'cmd')\s*:\s*("(?:\\.|[^"])*"|'(?:\\.|[^'])*')(\s*(?:,|\}))""")


def add_line_numbers(text):
    """py:2267-2276: every `cmd: 'x'` gets a `line: <its line number>` field (str.splitlines lines)."""
    out = []
    for i, line in enumerate(text.splitlines(keepends=True), start=1):
        out.append(_CMD.sub(lambda m: "%s:%s, line:%d%s" % (m.group(1), m.group(2), i, m.group(3)), line))
    return "".join(out)


def _simple_key(x):
    # get_simple_insertkey (py:477-495) on a task-list item; host glue, a loader runs once
    if type(x) != str:
        return None
    depth = 0
    for i, c in enumerate(x):
        if c == "}":
            depth -= 1
        if (depth == 0) != (i == 0 or i == len(x) - 1):
            return None
        if c == "{":
            depth += 1
    return x[1:-1]


def label_tasks(program):
    """py:1042-1072: `traceback_label` = '<cmd>-<line>' for every top-level and named task, and
    '<parent>/<cmd>-<line>' for nested `item` tasks and `tasks` lists (simple-insertkey entries
    are not tasks). Depth-first from the end of the list, like the reference's work list."""
    tasks = list(program["order"]) + list(program.get("named_tasks", {}).values())
    for t in tasks:
        if "line" not in t:
            raise JSON5Error("This task does not have a 'line' key: %r" % (t,))
        t["traceback_label"] = "%s-%s" % (t["cmd"], t["line"])
    todo = list(tasks)
    while todo:
        t = todo.pop()
        item = t.get("item", False)
        if item and isinstance(item, dict) and "cmd" in item:
            item["traceback_label"] = t["traceback_label"] + "/%s-%s" % (item["cmd"], item["line"])
            todo.append(item)
        if "tasks" in t:
            sub = t["tasks"]
            if _simple_key(sub):
                continue
            for st in sub:
                if _simple_key(st):
                    continue
                st["traceback_label"] = t["traceback_label"] + "/%s-%s" % (st["cmd"], st["line"])
            todo.extend(st for st in sub if not _simple_key(st))
    return program


def load_program(path_or_text, is_text=False):
    """py:2283-2312 for .json5 programs: -> (program, state). state = a copy of default_state with
    `output` defaulting to ''. The `tasks` -> `named_tasks` alias of rust-project/src/parser.rs:17-20
    is applied (the Python reference has no alias; math.json5 uses `tasks`)."""
    text = path_or_text if is_text else open(path_or_text, encoding="utf-8").read()
    program = loads(add_line_numbers(text))
    if not isinstance(program, dict) or "default_state" not in program:
        raise JSON5Error("a program is an object with 'default_state'")
    if "named_tasks" not in program and "tasks" in program:
        program["named_tasks"] = program.pop("tasks")
    program.setdefault("named_tasks", {})
    label_tasks(program)
    state = copy.deepcopy(program["default_state"])
    state["output"] = state.get("output", "")
    return program, state


class Runner:
    """The smallest interpreter loop that exercises the hot path the way the reference's does
    (py:2336-2405 -> py:1497-1501): every task passes through recursive_interpolate on the device
    before it runs. Commands beyond the plumbing set raise NotImplementedError: the interpreter
    is the caller of the hot path and out of scope.

    `resolve` is the batched recursive_interpolate of the mirror (device path); `on_interpolate`
    sees every string the pre-pass resolves (tests count them)."""

    COMMANDS = ("print", "set", "unescape", "label", "goto", "clear")

    def __init__(self, program, state, args=(), resolve=None, write=None):
        from . import interpolation_engine as IE
        self.IE = IE
        self.program = program
        self.state = state
        self.resolve = resolve or IE.recursive_interpolate
        self.write = write or (lambda s: None)
        if args:  # py:2343-2349, escaped on the device
            state["inserts"].update(IE.ingest_args(args))

    def step(self, task):
        inserts = self.state["inserts"]
        task = self.resolve(inserts, task)  # py:1501
        cmd = task.get("cmd")
        if cmd == "print":  # py:1669-1675 (the display unescape on the device)
            text = self.IE.display_text(task["text"])
            self.state["output"] += text
            self.write(text)
        elif cmd == "set":  # py:1657-1658
            inserts[task["output_name"]] = task["item"]
        elif cmd == "unescape":  # py:1660-1667
            inserts[task["output_name"]] = self.resolve(inserts, self.IE.recursive_unescape(task["item"]))
        elif cmd == "label":
            pass
        elif cmd == "goto":  # py:1685-1687
            if task["name"] != "CONTINUE":
                return {"goto_target": task["name"]}
        elif cmd == "clear":
            self.state["output"] = ""
        else:
            raise NotImplementedError("command %r is interpreter territory (out of scope)" % cmd)
        return None

    def run(self):
        order = self.program["order"]
        while self.state["order_index"] <= len(order):  # py:2359
            r = self.step(order[self.state["order_index"] - 1])
            if r is None:
                self.state["order_index"] += 1
            else:
                self.state["order_index"] = 2 + min(i for i, t in enumerate(order)
                                                     if t["cmd"] == "label" and t["name"] == r["goto_target"])
        return self.state["output"].strip()  # py:2403
