"""Siddhi QL front-end for the pattern / window hot path.

This is the stand-in for `siddhi-query-compiler` (ANTLR4 grammar
`QC/antlr4/io/siddhi/query/compiler/SiddhiQL.g4`) plus the variable-resolution half of
`CORE/util/parser/ExpressionParser.java:1255-1440`.  It parses the QL subset the hot path
covers and emits the *descriptor*: a JSON document that mirrors Siddhi's query-api AST
(`StateInputStream` / `StateElement` tree, `Selector`, `Partition`) with every variable
already resolved to (slot, chain-index, attribute, type) and every expression node carrying
its Java result type.  The descriptor is what crosses the C ABI (`include/siddhi_gfx.h`,
`sg_app_create`); the Java JNI shim would emit the same document from Siddhi's own parsed
`SiddhiApp`.

Supported subset (grammar line refs are to SiddhiQL.g4):
  * `@app:playback`, `@info(name=...)`, `define stream`            (:44-120)
  * `partition with (attr of S, ...) begin ... end`                  (:154-160)
  * single-stream queries with filters and `#window.length/time/lengthBatch` (:194-196)
  * pattern streams: every, ->, and/or, <n:m>, not S for T, within  (:200-289)
  * sequence streams: ',', +, *, ?, <n:m>                          (:291-353)
  * select / group by / having / limit / offset, sum avg count min max (:362-420)
  * insert into / return                                            (:425-440)
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

__all__ = ["parse_app", "compile_app", "SiddhiParserError", "TYPES"]

TYPES = ("STRING", "INT", "LONG", "FLOAT", "DOUBLE", "BOOL", "OBJECT")
ANY = -1  # SiddhiConstants.ANY  (CORE/util/SiddhiConstants.java:96)


class SiddhiParserError(Exception):
    pass


# --------------------------------------------------------------------------------------
# Lexer
# --------------------------------------------------------------------------------------
_TOKEN_RE = re.compile(r"""
    (?P<ws>\s+|--[^\n]*|/\*.*?\*/)
  | (?P<str>'[^']*'|"[^"]*")
  | (?P<num>(?:\d+\.\d*|\.\d+|\d+)(?:[eE][-+]?\d+)?[lLfFdD]?)
  | (?P<id>`[^`]*`|[A-Za-z_][A-Za-z_0-9]*)
  | (?P<op>->|<=|>=|==|!=|[-+*/%<>=!(),;\[\]#.:@?{}])
""", re.X | re.S)


@dataclass
class Tok:
    kind: str
    text: str
    pos: int

    @property
    def low(self) -> str:
        return self.text.lower()


def lex(src: str) -> List[Tok]:
    out, i = [], 0
    while i < len(src):
        m = _TOKEN_RE.match(src, i)
        if not m:
            raise SiddhiParserError(f"unexpected character {src[i]!r} at {i}")
        i = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        text = m.group(kind)
        if kind == "id" and text.startswith("`"):
            text = text[1:-1]
        out.append(Tok(kind, text, m.start()))
    out.append(Tok("eof", "", len(src)))
    return out


# --------------------------------------------------------------------------------------
# AST (mirrors io.siddhi.query.api)
# --------------------------------------------------------------------------------------
@dataclass
class Expr:
    op: str
    args: List[Any] = field(default_factory=list)
    # for vars: ref, index (None | int | ('last', k)), attr ; for const: type, value
    ref: Optional[str] = None
    index: Any = None
    attr: Optional[str] = None
    ctype: Optional[str] = None
    value: Any = None
    name: Optional[str] = None  # function name


@dataclass
class StreamEl:                       # StreamStateElement / AbsentStreamStateElement
    stream: str
    ref: Optional[str]
    filters: List[Expr]
    absent_wait: Optional[int] = None  # ms, for `not S for T`


@dataclass
class NextEl:
    a: Any
    b: Any


@dataclass
class EveryEl:
    e: Any


@dataclass
class LogicalEl:
    op: str  # AND / OR
    a: Any
    b: Any


@dataclass
class CountEl:
    e: StreamEl
    min: int
    max: int


@dataclass
class SingleInput:
    stream: str
    ref: Optional[str]
    handlers: List[Any]   # ("filter", Expr) | ("window", name, [Expr])


@dataclass
class StateInput:
    type: str             # PATTERN / SEQUENCE
    element: Any
    within: Optional[int]


@dataclass
class OutAttr:
    expr: Expr
    rename: Optional[str]


@dataclass
class Query:
    name: str
    input: Any
    select: Optional[List[OutAttr]]   # None => select *
    group_by: List[Expr]
    having: Optional[Expr]
    order_by: List[Any]
    limit: Optional[int]
    offset: Optional[int]
    output: Dict[str, Any]


@dataclass
class Partition:
    keys: Dict[str, str]   # stream -> attribute
    queries: List[Query]
    purge: Optional[Dict[str, int]] = None   # @purge(enable='true', interval, idle.period), in ms


# Expression.Time.timeToLong (siddhi-query-api Expression.java:250-306): the first digit run and the
# first non-digit run; units sec/min/hour/day/month/year only (no millisec)
_PURGE_UNITS = {"sec": 1000, "seconds": 1000, "second": 1000, "min": 60000, "minutes": 60000,
                "minute": 60000, "h": 3600000, "hour": 3600000, "hours": 3600000, "days": 86400000,
                "day": 86400000, "month": 30 * 86400000, "months": 30 * 86400000,
                "year": 365 * 86400000, "years": 365 * 86400000}


def _time_to_long(v: str) -> int:
    num = re.search(r"\d+", v)
    unit = re.search(r"\D+", v)
    if not num or not unit:
        raise SiddhiParserError(f"Provided retention value cannot be identified. retention period: {v}.")
    u = unit.group(0).strip().lower()
    if u not in _PURGE_UNITS:
        raise SiddhiParserError(f"Duration '{u}' does not exists ")
    return int(num.group(0)) * _PURGE_UNITS[u]


def _purge_of(annotations: List[Dict[str, Any]]) -> Optional[Dict[str, int]]:
    """PartitionRuntimeImpl constructor (:120-147): @purge needs `enable` ('true'/'false') and
    `idle.period`; `interval` defaults to 300000 ms.  None when absent or disabled."""
    for a in annotations:
        if a["name"] != "purge":
            continue
        el = {k.lower(): v for k, v in a["elements"].items()}
        if "enable" not in el:
            raise SiddhiParserError("Annotation @purge is missing element 'enable'")
        if el["enable"].lower() not in ("true", "false"):
            raise SiddhiParserError(f"Invalid value for enable: {el['enable']}. Please use 'true' or 'false'")
        if "idle.period" not in el:
            raise SiddhiParserError("Annotation @purge is missing element 'idle.period'")
        idle = _time_to_long(el["idle.period"])
        interval = _time_to_long(el["interval"]) if "interval" in el else 300000
        if el["enable"].lower() == "false":
            return None
        return {"interval": interval, "idle": idle}
    return None


@dataclass
class App:
    name: str
    playback: bool
    streams: Dict[str, List[List[str]]]
    queries: List[Query]
    partitions: List[Partition]
    order: List[Any] = field(default_factory=list)   # ("q" | "p", index): execution elements in app order


# --------------------------------------------------------------------------------------
# Parser
# --------------------------------------------------------------------------------------
_TIME_UNITS = [
    (re.compile(r"^years?$"), 365 * 86400000),
    (re.compile(r"^months?$"), 30 * 86400000),
    (re.compile(r"^weeks?$"), 7 * 86400000),
    (re.compile(r"^days?$"), 86400000),
    (re.compile(r"^hours?$"), 3600000),
    (re.compile(r"^min(ute|utes)?$"), 60000),
    (re.compile(r"^sec(ond|onds)?$"), 1000),
    (re.compile(r"^millisec(ond|onds)?$"), 1),
]


def _time_unit(word: str) -> Optional[int]:
    w = word.lower()
    for rx, ms in _TIME_UNITS:
        if rx.match(w):
            return ms
    return None


class Parser:
    def __init__(self, src: str):
        self.toks = lex(src)
        self.i = 0
        self.query_counter = 0

    # -- token helpers
    def peek(self, k: int = 0) -> Tok:
        return self.toks[min(self.i + k, len(self.toks) - 1)]

    def at(self, text: str, k: int = 0) -> bool:
        t = self.peek(k)
        if t.kind == "id":
            return t.low == text.lower()
        return t.text == text and t.kind in ("op",)

    def take(self) -> Tok:
        t = self.toks[self.i]
        self.i += 1
        return t

    def expect(self, text: str) -> Tok:
        if not self.at(text):
            t = self.peek()
            raise SiddhiParserError(f"expected {text!r} at {t.pos}, found {t.text!r}")
        return self.take()

    def accept(self, text: str) -> bool:
        if self.at(text):
            self.i += 1
            return True
        return False

    def nonneg_int(self, what: str) -> int:
        """`limit` / `offset` value: a non-negative integer (the reference refuses a negative one at
        creation, OrderByLimitTestCase.limitTest18/19)."""
        neg = self.accept("-")
        t = self.take()
        if neg or not t.text.isdigit():
            raise SiddhiParserError(f"{what} should be a non-negative integer, found {'-' if neg else ''}{t.text}")
        return int(t.text)

    def ident(self) -> str:
        t = self.peek()
        if t.kind != "id":
            raise SiddhiParserError(f"expected identifier at {t.pos}, found {t.text!r}")
        self.i += 1
        return t.text

    # -- app
    def parse_app(self) -> App:
        app = App(name="SiddhiApp", playback=False, streams={}, queries=[], partitions=[])
        pending_ann: List[Dict[str, Any]] = []
        while self.peek().kind != "eof":
            if self.accept(";"):
                continue
            if self.at("@"):
                pending_ann.append(self.parse_annotation())
                continue
            if self.at("define"):
                self.parse_define(app)
                pending_ann = []
                continue
            if self.at("partition"):
                app.partitions.append(self.parse_partition())
                app.partitions[-1].purge = _purge_of(pending_ann)
                app.order.append(("p", len(app.partitions) - 1))
                pending_ann = []
                continue
            if self.at("from"):
                app.queries.append(self.parse_query(pending_ann))
                app.order.append(("q", len(app.queries) - 1))
                pending_ann = []
                continue
            raise SiddhiParserError(f"unexpected token {self.peek().text!r} at {self.peek().pos}")
        return app

    def parse_annotation(self) -> Dict[str, Any]:
        self.expect("@")
        name = self.ident()
        if self.accept(":"):
            name = name + ":" + self.ident()
        elems: Dict[str, Any] = {}
        if self.accept("("):
            idx = 0
            while not self.at(")"):
                # element keys may be dotted (`idle.period`)
                k = 0
                while self.peek(k).kind == "id" and self.at(".", k + 1):
                    k += 2
                if self.peek(k).kind == "id" and self.at("=", k + 1):
                    key = self.ident()
                    while self.accept("."):
                        key += "." + self.ident()
                    self.expect("=")
                else:
                    key = f"_{idx}"
                t = self.take()
                elems[key] = t.text[1:-1] if t.kind == "str" else t.text
                idx += 1
                self.accept(",")
            self.expect(")")
        ann = {"name": name.lower(), "elements": elems}
        if ann["name"] in ("app:playback",):
            self._app_playback = True
        if ann["name"] == "app:name":
            self._app_name = elems.get("_0")
        return ann

    def parse_define(self, app: App) -> None:
        self.expect("define")
        kind = self.ident().lower()
        if kind != "stream":
            raise SiddhiParserError(f"only 'define stream' is supported on this path (got {kind})")
        name = self.ident()
        self.expect("(")
        attrs = []
        while True:
            an = self.ident()
            at = self.ident().upper()
            if at not in TYPES:
                raise SiddhiParserError(f"unknown attribute type {at}")
            attrs.append([an, at])
            if not self.accept(","):
                break
        self.expect(")")
        app.streams[name] = attrs

    def parse_partition(self) -> Partition:
        self.expect("partition")
        self.expect("with")
        self.expect("(")
        keys = {}
        while True:
            attr = self.ident()
            self.expect("of")
            stream = self.ident()
            keys[stream] = attr
            if not self.accept(","):
                break
        self.expect(")")
        self.expect("begin")
        queries = []
        pending: List[Dict[str, Any]] = []
        while not self.at("end"):
            if self.accept(";"):
                continue
            if self.at("@"):
                pending.append(self.parse_annotation())
                continue
            queries.append(self.parse_query(pending))
            pending = []
        self.expect("end")
        return Partition(keys=keys, queries=queries)

    # -- query
    def parse_query(self, annotations: List[Dict[str, Any]]) -> Query:
        name = None
        for a in annotations:
            if a["name"] == "info":
                name = a["elements"].get("name", a["elements"].get("_0"))
        self.query_counter += 1
        if name is None:
            name = f"query_{self.query_counter}"
        self.expect("from")
        inp = self.parse_query_input()
        select = None
        group_by: List[Expr] = []
        having = None
        order_by: List[Any] = []
        limit = offset = None
        if self.accept("select"):
            if self.accept("*"):
                select = None
            else:
                select = []
                while True:
                    e = self.parse_expr()
                    rename = None
                    if self.accept("as"):
                        rename = self.ident()
                    select.append(OutAttr(e, rename))
                    if not self.accept(","):
                        break
        if self.at("group"):
            self.take()
            self.expect("by")
            while True:
                group_by.append(self.parse_expr())
                if not self.accept(","):
                    break
        if self.accept("having"):
            having = self.parse_expr()
        if self.at("order"):
            self.take()
            self.expect("by")
            while True:
                v = self.parse_expr()
                direction = "asc"
                if self.at("asc") or self.at("desc"):
                    direction = self.take().low
                order_by.append((v, direction))
                if not self.accept(","):
                    break
        if self.accept("limit"):
            limit = self.nonneg_int("limit")
        if self.accept("offset"):
            offset = self.nonneg_int("offset")
        output: Dict[str, Any]
        if self.accept("insert"):
            events = "current"
            if self.at("current") or self.at("expired") or self.at("all"):
                events = self.take().low
                self.expect("events")
            else:
                self.accept("events")   # `insert events into` = current events (SiddhiQL.g4 output_event_type)
            self.expect("into")
            output = {"kind": "insert", "stream": self.ident(), "events": events}
        elif self.accept("return"):
            events = "current"
            if self.at("current") or self.at("expired") or self.at("all"):
                events = self.take().low
                self.expect("events")
            output = {"kind": "return", "events": events}
        else:
            output = {"kind": "return", "events": "current"}
        return Query(name=name, input=inp, select=select, group_by=group_by, having=having,
                     order_by=order_by, limit=limit, offset=offset, output=output)

    def _is_state_input(self) -> bool:
        """Scan ahead (bracket-aware) to decide if the input is a pattern/sequence."""
        depth = 0
        j = self.i
        while True:
            t = self.toks[j]
            if t.kind == "eof":
                return False
            if t.kind == "op" and t.text in "([":
                depth += 1
            elif t.kind == "op" and t.text in ")]":
                depth -= 1
            elif depth <= 0 and t.kind == "id" and t.low in ("select", "insert", "return",
                                                              "group", "having", "order",
                                                              "limit", "output"):
                return False
            elif depth <= 0 and t.kind == "op" and t.text == ";":
                return False
            if t.kind == "op" and t.text in ("->",):
                return True
            if t.kind == "id" and t.low in ("every", "within", "not"):
                return True
            if depth == 0 and t.kind == "op" and t.text == "=" and self.toks[j - 1].kind == "id" \
                    and not (self.toks[j - 2].kind == "op" and self.toks[j - 2].text in ("<", ">", "!", "=")):
                return True
            if depth == 0 and t.kind == "op" and t.text == ",":
                return True
            if depth == 0 and t.kind == "op" and t.text in ("+", "*", "?") and \
                    self.toks[j - 1].kind == "op" and self.toks[j - 1].text == "]":
                return True
            if depth == 0 and t.kind == "op" and t.text == "<" and self.toks[j + 1].kind == "num":
                return True
            if depth == 0 and t.kind == "id" and t.low in ("and", "or"):
                return True
            j += 1

    def parse_query_input(self):
        if self._is_state_input():
            return self.parse_state_input()
        stream = self.ident()
        ref = None
        if self.accept("as"):
            ref = self.ident()
        handlers = self.parse_handlers(allow_window=True)
        return SingleInput(stream=stream, ref=ref, handlers=handlers)

    def parse_handlers(self, allow_window: bool) -> List[Any]:
        hs: List[Any] = []
        while True:
            if self.at("["):
                self.take()
                hs.append(("filter", self.parse_expr()))
                self.expect("]")
            elif self.at("#") and self.at("[", 1):
                self.take(); self.take()
                hs.append(("filter", self.parse_expr()))
                self.expect("]")
            elif self.at("#") and self.peek(1).kind == "id" and self.peek(1).low == "window":
                if not allow_window:
                    raise SiddhiParserError("windows are not allowed inside pattern/sequence sources "
                                            "(SiddhiQL.g4:287-289)")
                self.take(); self.take(); self.expect(".")
                wname = self.ident()
                self.expect("(")
                params = []
                while not self.at(")"):
                    params.append(self.parse_expr())
                    self.accept(",")
                self.expect(")")
                hs.append(("window", wname, params))
            else:
                return hs

    # -- pattern / sequence
    def parse_state_input(self) -> StateInput:
        # Decide PATTERN vs SEQUENCE: a top-level ',' means sequence.
        depth, j, seq = 0, self.i, False
        while True:
            t = self.toks[j]
            if t.kind == "eof":
                break
            if t.kind == "op" and t.text in "([":
                depth += 1
            elif t.kind == "op" and t.text in ")]":
                depth -= 1
            elif t.kind == "op" and t.text == ";":
                break
            elif t.kind == "id" and t.low in ("select", "insert", "return", "within") and depth == 0:
                break
            elif t.kind == "op" and t.text == "," and depth == 0:
                seq = True
            elif t.kind == "op" and t.text == "->":
                seq = False
                break
            j += 1
        self.seq = seq
        el = self.parse_chain()
        within = None
        if self.accept("within"):
            within = self.parse_time_value()
        return StateInput(type="SEQUENCE" if seq else "PATTERN", element=el, within=within)

    def parse_time_value(self) -> int:
        total = 0
        got = False
        while self.peek().kind == "num" and self.peek(1).kind == "id" and _time_unit(self.peek(1).text):
            n = int(self.take().text)
            total += n * _time_unit(self.take().text)
            got = True
        if not got:
            raise SiddhiParserError(f"expected time value at {self.peek().pos}")
        return total

    def parse_chain(self):
        sep = "," if self.seq else "->"
        left = self.parse_chain_item()
        while self.at(sep):
            self.take()
            right = self.parse_chain_item()
            left = NextEl(left, right)   # left-associative (ANTLR4 left recursion)
        return left

    def parse_chain_item(self):
        if self.accept("every"):
            if self.at("("):
                return EveryEl(self.parse_paren_chain())
            return EveryEl(self.parse_source())
        if self.at("(") and not self._paren_is_logical_absent():
            return self.parse_paren_chain()
        return self.parse_source()

    def _paren_is_logical_absent(self) -> bool:
        return False

    def parse_paren_chain(self):
        self.expect("(")
        el = self.parse_chain()
        self.expect(")")
        return el

    def parse_source(self):
        """pattern_source: logical | collection | standard | absent  (SiddhiQL.g4:258-262)."""
        a = self.parse_stateful_or_absent()
        if self.at("and") or self.at("or"):
            op = self.take().low.upper()
            b = self.parse_stateful_or_absent()
            return LogicalEl(op, a, b)
        return a

    def parse_stateful_or_absent(self):
        if self.accept("not"):
            stream = self.ident()
            filters = [h[1] for h in self.parse_handlers(allow_window=False)]
            if self.accept("for"):
                wait = self.parse_time_value()
            else:
                wait = None   # `A and not B` form: absent without waiting time
            return StreamEl(stream, None, filters, absent_wait=wait if wait is not None else -1)
        ref = None
        if self.peek().kind == "id" and self.at("=", 1):
            ref = self.ident()
            self.expect("=")
        stream = self.ident()
        filters = [h[1] for h in self.parse_handlers(allow_window=False)]
        el = StreamEl(stream, ref, filters)
        # collections  <n:m>  (pattern) ; + * ? <n:m> (sequence)
        if self.at("<") and (self.peek(1).kind == "num" or self.at(":", 1)):
            self.take()
            mn, mx = ANY, ANY
            if self.accept(":"):
                mx = int(self.take().text)
            else:
                mn = int(self.take().text)
                if self.accept(":"):
                    if self.peek().kind == "num":
                        mx = int(self.take().text)
                else:
                    mx = mn
            self.expect(">")
            return CountEl(el, mn, mx)
        if self.seq:
            if self.accept("+"):
                return CountEl(el, 1, ANY)
            if self.accept("*"):
                return CountEl(el, 0, ANY)
            if self.accept("?"):
                return CountEl(el, 0, 1)
        return el

    # -- expressions (precedence per SiddhiQL.g4 math_operation)
    def parse_expr(self) -> Expr:
        return self.parse_or()

    def parse_or(self):
        l = self.parse_and()
        while self.at("or"):
            self.take()
            l = Expr("or", [l, self.parse_and()])
        return l

    def parse_and(self):
        l = self.parse_eq()
        while self.at("and"):
            self.take()
            l = Expr("and", [l, self.parse_eq()])
        return l

    def parse_eq(self):
        l = self.parse_cmp()
        while self.at("==") or self.at("!="):
            op = self.take().text
            l = Expr(op, [l, self.parse_cmp()])
        return l

    def parse_cmp(self):
        l = self.parse_add()
        while self.at(">=") or self.at("<=") or self.at(">") or self.at("<"):
            op = self.take().text
            l = Expr(op, [l, self.parse_add()])
        return l

    def parse_add(self):
        l = self.parse_mul()
        while self.at("+") or self.at("-"):
            op = self.take().text
            l = Expr(op, [l, self.parse_mul()])
        return l

    def parse_mul(self):
        l = self.parse_unary()
        while self.at("*") or self.at("/") or self.at("%"):
            op = self.take().text
            l = Expr(op, [l, self.parse_unary()])
        return l

    def parse_unary(self):
        if self.accept("not"):
            return Expr("not", [self.parse_unary()])
        if self.at("-") and self.peek(1).kind == "num":
            self.take()
            return self._number(self.take().text, negate=True)
        if self.at("+") and self.peek(1).kind == "num":
            self.take()
        return self.parse_primary()

    def _number(self, text: str, negate: bool = False) -> Expr:
        s = -1 if negate else 1
        suf = text[-1].lower()
        if suf == "l":
            return Expr("const", ctype="LONG", value=s * int(text[:-1]))
        if suf == "f":
            return Expr("const", ctype="FLOAT", value=s * float(text[:-1]))
        if suf == "d":
            return Expr("const", ctype="DOUBLE", value=s * float(text[:-1]))
        if re.fullmatch(r"\d+", text):
            return Expr("const", ctype="INT", value=s * int(text))
        return Expr("const", ctype="DOUBLE", value=s * float(text))

    def parse_primary(self) -> Expr:
        t = self.peek()
        if self.accept("("):
            e = self.parse_expr()
            self.expect(")")
            return e
        if t.kind == "num":
            # time constant?
            if self.peek(1).kind == "id" and _time_unit(self.peek(1).text):
                return Expr("const", ctype="LONG", value=self.parse_time_value())
            self.take()
            return self._number(t.text)
        if t.kind == "str":
            self.take()
            return Expr("const", ctype="STRING", value=t.text[1:-1])
        if t.kind == "id":
            if t.low in ("true", "false"):
                self.take()
                return Expr("const", ctype="BOOL", value=(t.low == "true"))
            if t.low == "null":
                self.take()
                return Expr("const", ctype="OBJECT", value=None)
            name = self.ident()
            if self.at("("):
                self.take()
                args = []
                while not self.at(")"):
                    args.append(self.parse_expr())
                    self.accept(",")
                self.expect(")")
                e = Expr("fn", args, name=name)
            else:
                index = None
                if self.at("["):
                    self.take()
                    if self.accept("last"):
                        k = 0
                        if self.accept("-"):
                            k = int(self.take().text)
                        index = ("last", k)
                    else:
                        index = int(self.take().text)
                    self.expect("]")
                if self.accept("."):
                    attr = self.ident()
                    e = Expr("var", ref=name, index=index, attr=attr)
                else:
                    e = Expr("var", ref=None, index=index, attr=name)
            if self.at("is") and self.at("null", 1):
                self.take(); self.take()
                return Expr("isnull", [e])
            return e
        raise SiddhiParserError(f"unexpected token {t.text!r} at {t.pos}")


def parse_app(src: str) -> App:
    p = Parser(src)
    p._app_playback = False
    p._app_name = None
    app = p.parse_app()
    app.playback = p._app_playback
    if p._app_name:
        app.name = p._app_name
    return app


# --------------------------------------------------------------------------------------
# Resolution: AST -> descriptor JSON (typed, slot-resolved)
# --------------------------------------------------------------------------------------
_NUM_RANK = {"INT": 0, "LONG": 1, "FLOAT": 2, "DOUBLE": 3}
_AGGS = {"sum", "avg", "count", "min", "max", "distinctcount", "stddev", "maxforever", "minforever"}


def _promote(a: str, b: str) -> str:
    """JLS §5.6.2 binary numeric promotion as Siddhi's executor factories apply it."""
    if a not in _NUM_RANK or b not in _NUM_RANK:
        raise SiddhiParserError(f"arithmetic on non-numeric types {a}, {b}")
    return a if _NUM_RANK[a] >= _NUM_RANK[b] else b


class Resolver:
    """Resolves variables the way ExpressionParser.parseVariable does.

    For a state query `slots` is the MetaStateEvent order: a list of (stream, ref, multi).
    For a single-stream query `slots` has a single entry and slot index -1 is used.
    """

    def __init__(self, streams, slots, single: bool, out_attrs: Optional[List[List[str]]] = None):
        self.streams = streams
        self.slots = slots
        self.single = single
        self.out_attrs = out_attrs or []

    def attr_of(self, stream: str, attr: str):
        for i, (an, at) in enumerate(self.streams[stream]):
            if an == attr:
                return i, at
        return None

    def var(self, e: Expr, current_state: Optional[int], default_index: int, having: bool = False):
        # HAVING: output-stream attributes first (ExpressionParser.java:1316-1323)
        if having and e.ref is None:
            for i, (an, at) in enumerate(self.out_attrs):
                if an == e.attr:
                    return {"op": "outvar", "attr": i, "t": at}
        if self.single:
            stream = self.slots[0][0]
            if e.ref is not None and e.ref not in (stream, self.slots[0][1]):
                raise SiddhiParserError(f"Id '{e.ref}' not defined within the current scope")
            r = self.attr_of(stream, e.attr)
            if r is None:
                raise SiddhiParserError(f"attribute {e.attr} not found in {stream}")
            return {"op": "var", "slot": -1, "chain": 0, "attr": r[0], "t": r[1]}
        # index in chain (ExpressionParser.java:1262-1270)
        idx = e.index
        if idx is None:
            chain = default_index
        elif isinstance(idx, tuple):
            raw = -2 - idx[1]                 # LAST = -2, last-k = -2-k
            chain = raw + 1
        else:
            chain = idx
        slot = None
        t = None
        multi = False
        if e.ref is None:
            if current_state is not None and current_state >= 0:
                stream = self.slots[current_state][0]
                r = self.attr_of(stream, e.attr)
                if r is None:
                    raise SiddhiParserError(f"attribute {e.attr} not in stream {stream}")
                slot, (ai, t) = current_state, r
            else:
                found = None
                for i, (stream, ref, _m) in enumerate(self.slots):
                    r = self.attr_of(stream, e.attr)
                    if r is not None:
                        if found is not None:
                            raise SiddhiParserError(f"attribute '{e.attr}' is ambiguous")
                        found = (i, r)
                if found is None:
                    raise SiddhiParserError(f"No matching stream reference found for attribute '{e.attr}'")
                slot, (ai, t) = found[0], found[1]
        else:
            for i, (stream, ref, m) in enumerate(self.slots):
                if (ref is None and stream == e.ref) or (ref is not None and ref == e.ref):
                    r = self.attr_of(stream, e.attr)
                    if r is None:
                        raise SiddhiParserError(f"attribute {e.attr} not in stream {stream}")
                    slot, (ai, t) = i, r
                    if current_state is not None and current_state > -1 and \
                            self.slots[current_state][1] is not None and isinstance(idx, tuple):
                        if e.ref == self.slots[current_state][1]:
                            chain = -2 - idx[1]          # own-state [last] keeps the raw index
                    elif current_state is None and idx is None:
                        multi = m
                    break
            if slot is None:
                raise SiddhiParserError(f"Stream with reference '{e.ref}' not found for attribute '{e.attr}'")
        d = {"op": "var", "slot": slot, "chain": chain, "attr": ai, "t": t}
        if multi:
            return {"op": "multivar", "slot": slot, "attr": ai, "t": "OBJECT"}
        return d

    def expr(self, e: Expr, current_state: Optional[int], default_index: int,
             having: bool = False, allow_agg: bool = False) -> Dict[str, Any]:
        op = e.op
        if op == "const":
            return {"op": "const", "t": e.ctype, "v": e.value}
        if op == "var":
            return self.var(e, current_state, default_index, having)
        if op in ("and", "or"):
            a = self.expr(e.args[0], current_state, default_index, having, allow_agg)
            b = self.expr(e.args[1], current_state, default_index, having, allow_agg)
            return {"op": op, "a": a, "b": b, "t": "BOOL"}
        if op == "not":
            a = self.expr(e.args[0], current_state, default_index, having, allow_agg)
            return {"op": "not", "a": a, "t": "BOOL"}
        if op == "isnull":
            a = self.expr(e.args[0], current_state, default_index, having, allow_agg)
            return {"op": "isnull", "a": a, "t": "BOOL"}
        if op in (">", "<", ">=", "<=", "==", "!="):
            a = self.expr(e.args[0], current_state, default_index, having, allow_agg)
            b = self.expr(e.args[1], current_state, default_index, having, allow_agg)
            ta, tb = a["t"], b["t"]
            if op in ("==", "!=") and (ta in ("STRING", "BOOL") or tb in ("STRING", "BOOL")):
                if ta != tb and "OBJECT" not in (ta, tb):
                    raise SiddhiParserError(f"cannot compare {ta} with {tb}")
                ct = ta if ta != "OBJECT" else tb
            elif ta == "OBJECT" or tb == "OBJECT":
                ct = "OBJECT"
            else:
                ct = _promote(ta, tb)
            return {"op": op, "a": a, "b": b, "ct": ct, "t": "BOOL"}
        if op in ("+", "-", "*", "/", "%"):
            a = self.expr(e.args[0], current_state, default_index, having, allow_agg)
            b = self.expr(e.args[1], current_state, default_index, having, allow_agg)
            return {"op": op, "a": a, "b": b, "t": _promote(a["t"], b["t"])}
        if op == "fn":
            name = e.name.lower()
            if name in _AGGS:
                if not allow_agg:
                    raise SiddhiParserError(f"aggregator {name} not allowed here")
                args = [self.expr(x, current_state, default_index, having, False) for x in e.args]
                if len(args) > 1 or (name != "count" and len(args) != 1):
                    # e.g. SumAttributeAggregatorExecutor.init: exactly 1 parameter (count: 0 or 1)
                    raise SiddhiParserError(f"{name} aggregator has to have exactly 1 parameter, currently "
                                            f"{len(args)} parameters provided")
                if name in ("sum", "avg", "stddev", "min", "max", "minforever", "maxforever") and \
                        args[0]["t"] not in ("INT", "LONG", "FLOAT", "DOUBLE"):
                    # e.g. SumAttributeAggregatorExecutor.init: OperationNotSupportedException for other types
                    raise SiddhiParserError(f"{name} not supported for {args[0]['t']}")
                if name == "count":
                    t = "LONG"
                elif name == "avg":
                    t = "DOUBLE"
                elif name == "sum":
                    at = args[0]["t"]
                    t = "LONG" if at in ("INT", "LONG") else "DOUBLE"
                elif name in ("min", "max", "minforever", "maxforever"):
                    t = args[0]["t"]
                elif name == "distinctcount":
                    t = "LONG"
                else:
                    t = "DOUBLE"
                return {"op": "agg", "name": name, "args": args, "t": t}
            raise SiddhiParserError(f"function {e.name} is not supported on this path")
        raise SiddhiParserError(f"unsupported expression {op}")


def _slot_order(el, out: List):
    """MetaStateEvent order = order SingleInputStreamParser is invoked in
    StateInputStreamParser.parse (Next: current then next; Logical: element2 then element1)."""
    if isinstance(el, StreamEl):
        out.append(el)
    elif isinstance(el, NextEl):
        _slot_order(el.a, out); _slot_order(el.b, out)
    elif isinstance(el, EveryEl):
        _slot_order(el.e, out)
    elif isinstance(el, LogicalEl):
        _slot_order(el.b, out); _slot_order(el.a, out)
    elif isinstance(el, CountEl):
        _slot_order(el.e, out)
    return out


def _element_json(el, slot_of, resolver: Resolver, multi_slots):
    if isinstance(el, StreamEl):
        s = slot_of[id(el)]
        d = {"k": "absent" if el.absent_wait is not None else "stream", "stream": el.stream,
             "slot": s,
             "filters": [resolver.expr(f, s, -1) for f in el.filters]}
        if el.absent_wait is not None:
            d["wait"] = el.absent_wait
        return d
    if isinstance(el, NextEl):
        return {"k": "next", "a": _element_json(el.a, slot_of, resolver, multi_slots),
                "b": _element_json(el.b, slot_of, resolver, multi_slots)}
    if isinstance(el, EveryEl):
        return {"k": "every", "e": _element_json(el.e, slot_of, resolver, multi_slots)}
    if isinstance(el, LogicalEl):
        return {"k": "logical", "op": el.op, "a": _element_json(el.a, slot_of, resolver, multi_slots),
                "b": _element_json(el.b, slot_of, resolver, multi_slots)}
    if isinstance(el, CountEl):
        return {"k": "count", "min": el.min, "max": el.max,
                "e": _element_json(el.e, slot_of, resolver, multi_slots)}
    raise SiddhiParserError("bad state element")


def _selector_json(q: Query, streams, resolver: Resolver, input_attrs: List[List[str]]):
    attrs = []
    if q.select is None:   # select *
        if resolver.single:
            for i, (an, at) in enumerate(input_attrs):
                attrs.append({"name": an, "e": {"op": "var", "slot": -1, "chain": 0, "attr": i, "t": at}})
        else:
            for si, (stream, ref, _m) in enumerate(resolver.slots):
                for i, (an, at) in enumerate(streams[stream]):
                    attrs.append({"name": an, "e": {"op": "var", "slot": si, "chain": 0, "attr": i, "t": at}})
    else:
        for oa in q.select:
            name = oa.rename
            if name is None:
                if oa.expr.op == "var":
                    name = oa.expr.attr
                else:
                    raise SiddhiParserError("output attribute needs a name ('as ...')")
            attrs.append({"name": name, "e": resolver.expr(oa.expr, None, 0, allow_agg=True)})
    out_attrs = [[a["name"], a["e"]["t"]] for a in attrs]
    resolver.out_attrs = out_attrs
    sel = {"attrs": attrs,
           "group_by": [resolver.expr(g, None, 0) for g in q.group_by],
           "having": resolver.expr(q.having, None, 0, having=True, allow_agg=True) if q.having else None,
           "order_by": [[resolver.expr(v, None, 0, having=True), d] for v, d in q.order_by],
           "limit": q.limit, "offset": q.offset}
    return sel, out_attrs


def _check_window(name: str, params: List[Dict[str, Any]]):
    """Creation-time parameter checks of the windows (SiddhiAppValidationException in the reference):
    LengthWindowProcessor.init (one constant int), TimeWindowProcessor.init (one constant int/long),
    LengthBatchWindowProcessor.init :125-147 (constant int length, optional constant bool
    stream.current.event, at most two)."""
    def const(p, types):
        return p.get("op") == "const" and p.get("t") in types
    n = name.lower()
    if n == "length":
        if len(params) != 1 or not const(params[0], ("INT",)):
            raise SiddhiParserError(f"Length window should only have one parameter (<int> windowLength), "
                                    f"but found {len(params)} input parameters")
    elif n == "time":
        if len(params) != 1 or not const(params[0], ("INT", "LONG")):
            raise SiddhiParserError("Time window should only have one constant int or long parameter "
                                    f"(<int|long|time> windowTime), but found {len(params)} input parameters")
    elif n == "lengthbatch":
        if not 1 <= len(params) <= 2:
            raise SiddhiParserError("LengthBatch window should have one parameter (<int> window.length) or two "
                                    "parameters (<int> window.length, <bool> stream.current.event), but found "
                                    f"{len(params)} input parameters.")
        if not const(params[0], ("INT",)):
            raise SiddhiParserError("LengthBatch window's window.length parameter should be a constant int")
        if len(params) == 2 and not const(params[1], ("BOOL",)):
            raise SiddhiParserError("LengthBatch window's stream.current.event parameter should be a constant bool")


def _query_json(q: Query, app: App, partition_keys: Optional[Dict[str, str]], part: Optional[int] = None,
                purge: Optional[Dict[str, int]] = None):
    streams = dict(app.streams)
    if isinstance(q.input, SingleInput):
        if q.input.stream not in streams:
            raise SiddhiParserError(f"stream {q.input.stream} is not defined")
        res = Resolver(streams, [(q.input.stream, q.input.ref, False)], single=True)
        handlers = []
        for h in q.input.handlers:
            if h[0] == "filter":
                handlers.append({"k": "filter", "e": res.expr(h[1], -1, -1)})
            else:
                params = [res.expr(p, -1, -1) for p in h[2]]
                _check_window(h[1], params)
                handlers.append({"k": "window", "name": h[1], "params": params})
        sel, out_attrs = _selector_json(q, streams, res, streams[q.input.stream])
        inp = {"kind": "single", "stream": q.input.stream, "handlers": handlers}
    else:
        els = _slot_order(q.input.element, [])
        multi = set()

        def mark(el, in_count=False):
            if isinstance(el, StreamEl) and in_count:
                multi.add(id(el))
            elif isinstance(el, NextEl):
                mark(el.a); mark(el.b)
            elif isinstance(el, EveryEl):
                mark(el.e)
            elif isinstance(el, LogicalEl):
                mark(el.a); mark(el.b)
            elif isinstance(el, CountEl):
                mark(el.e, True)
        mark(q.input.element)
        for e in els:
            if e.stream not in streams:
                raise SiddhiParserError(f"stream {e.stream} is not defined")
        slots = [(e.stream, e.ref, id(e) in multi) for e in els]
        slot_of = {id(e): i for i, e in enumerate(els)}
        res = Resolver(streams, slots, single=False)
        element = _element_json(q.input.element, slot_of, res, multi)
        sel, out_attrs = _selector_json(q, streams, res, [])
        inp = {"kind": "state", "type": q.input.type, "within": q.input.within,
               "element": element,
               "slots": [{"stream": s, "ref": r, "multi": m} for s, r, m in slots]}
    d = {"name": q.name, "input": inp, "select": sel, "output": q.output, "out_attrs": out_attrs}
    if partition_keys is not None:
        keyed = {}
        for s, a in partition_keys.items():
            r = [i for i, (an, _t) in enumerate(streams[s]) if an == a]
            if not r:
                raise SiddhiParserError(f"partition key {a} not in {s}")
            keyed[s] = r[0]
        d["partition"] = keyed
        d["partition_id"] = part
        if purge:
            d["purge"] = dict(purge)
    return d


def compile_app(src: str) -> Dict[str, Any]:
    """QL text -> descriptor dict (JSON-serialisable)."""
    app = parse_app(src)
    queries = []

    def add(q, keys, part=None, purge=None):
        d = _query_json(q, app, keys, part, purge)
        queries.append(d)
        # an `insert into` target that is not defined becomes a defined stream
        # (SiddhiAppParser defines output streams from the selector's output attributes)
        if d["output"]["kind"] == "insert" and d["output"]["stream"] not in app.streams:
            app.streams[d["output"]["stream"]] = [list(a) for a in d["out_attrs"]]

    # execution elements in app order: the order SiddhiAppRuntimeBuilder subscribes them
    for kind, i in app.order:
        if kind == "q":
            add(app.queries[i], None)
        else:
            for q in app.partitions[i].queries:
                add(q, app.partitions[i].keys, i, app.partitions[i].purge)
    return {"version": 1, "name": app.name, "playback": app.playback,
            "streams": app.streams, "queries": queries}


def descriptor_json(src: str) -> str:
    return json.dumps(compile_app(src), separators=(",", ":"))
