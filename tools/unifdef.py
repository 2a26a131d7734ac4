#!/usr/bin/env python3
"""A small unifdef: resolve preprocessor conditionals over named macros in place, keeping the code of the
branch the default build compiles (used to prune A/B options out of csrc/ with the product code objects
unchanged, profiles/r06/README.md).

  -D NAME=VALUE   the macro is defined with VALUE in the default build (its `#ifndef NAME / #define NAME v /
                  #endif` guard is dropped WITH the define: the macro only steered conditionals)
  -K NAME=VALUE   as -D, but the guard's `#define` line is kept, unconditionally (a tunable the code reads)
  -U NAME         the macro is undefined in the default build

A conditional whose expression still names an unresolved identifier after substitution is kept (its
branches are still processed).  Prints the resolved-away count and any -D / -U name left in the text.

usage: python tools/unifdef.py FILE [-D N=V ...] [-K N=V ...] [-U N ...]
"""
from __future__ import annotations

import argparse
import re
import sys

DIRECTIVE = re.compile(r"^\s*#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)$")
IDENT = re.compile(r"\b[A-Za-z_]\w*\b")


def _strip_comment(s: str) -> str:
    return re.sub(r"//.*$", "", re.sub(r"/\*.*?\*/", "", s)).strip()


def evaluate(kind: str, arg: str, defs: dict, undefs: set):
    """True / False, or None when the condition names a macro outside defs / undefs."""
    arg = _strip_comment(arg)
    if kind in ("ifdef", "ifndef"):
        name = arg.split()[0]
        if name in defs:
            v = True
        elif name in undefs:
            v = False
        else:
            return None
        return v if kind == "ifdef" else not v

    def repl_defined(m):
        n = m.group(1)
        if n in defs:
            return "1"
        if n in undefs:
            return "0"
        return m.group(0)
    e = re.sub(r"\bdefined\s*\(\s*(\w+)\s*\)", repl_defined, arg)
    e = re.sub(r"\bdefined\s+(\w+)", repl_defined, e)
    for _ in range(8):                                    # macro values may name other macros
        e2 = IDENT.sub(lambda m: f"({defs[m.group(0)]})" if m.group(0) in defs else
                       ("0" if m.group(0) in undefs else m.group(0)), e)
        if e2 == e:
            break
        e = e2
    if IDENT.search(e.replace("and", "").replace("or", "").replace("not", "")):
        return None
    py = e.replace("&&", " and ").replace("||", " or ")
    py = re.sub(r"!(?!=)", " not ", py)
    py = re.sub(r"(\d+)[uUlL]+\b", r"\1", py)
    try:
        return bool(eval(py, {"__builtins__": {}}, {}))     # noqa: S307 (integer expressions of -D values)
    except Exception:
        return None


def process(lines: list[str], defs: dict, keep: set, undefs: set) -> tuple[list[str], int]:
    out: list[str] = []
    # frame per open conditional: resolved (bool: this conditional's directives are dropped), emit (bool: the
    # current branch's lines are emitted), taken (a known-true branch was seen), emitted_directive (an
    # unresolved #if / #elif was kept, so #else / #endif must be kept too), parent_emit
    stack: list[dict] = []
    removed = 0
    i = 0

    def emitting() -> bool:
        return all(f["emit"] for f in stack)

    while i < len(lines):
        ln = lines[i]
        m = DIRECTIVE.match(ln)
        if not m:
            if emitting():
                out.append(ln)
            i += 1
            continue
        kind, arg = m.group(1), m.group(2)
        if kind in ("if", "ifdef", "ifndef"):
            v = evaluate(kind, arg, defs, undefs) if emitting() else None
            if not emitting():
                stack.append({"emit": False, "taken": True, "kept": False, "skip": True})
                i += 1
                continue
            # the `#ifndef X / #define X v / #endif` guard of a -K tunable: keep the define, drop the guard
            if kind == "ifndef" and v is False and arg.split()[0] in keep:
                name = arg.split()[0]
                j = i + 1
                body = []
                while not DIRECTIVE.match(lines[j]):
                    body.append(lines[j])
                    j += 1
                if DIRECTIVE.match(lines[j]).group(1) == "endif" and any(
                        re.match(rf"\s*#\s*define\s+{name}\b", b) for b in body):
                    out.extend(body)
                    removed += 1
                    i = j + 1
                    continue
            if v is None:
                out.append(ln)
                stack.append({"emit": True, "taken": False, "kept": True, "skip": False})
            else:
                removed += 1
                stack.append({"emit": v, "taken": v, "kept": False, "skip": False})
            i += 1
            continue
        f = stack[-1] if stack else None
        if f is None:
            raise SystemExit(f"unbalanced #{kind} at line {i + 1}")
        if f["skip"]:                          # inside a branch that is not emitted: track nesting only
            if kind == "endif":
                stack.pop()
            i += 1
            continue
        if kind == "elif":
            if f["taken"]:
                f["emit"] = False
            else:
                v = evaluate("if", arg, defs, undefs)
                if v is None:
                    out.append(ln.replace("#elif", "#if", 1) if not f["kept"] else ln)
                    f["kept"] = True
                    f["emit"] = True
                elif v:
                    if f["kept"]:
                        out.append(re.sub(r"#\s*elif.*", "#else", ln))
                    f["emit"], f["taken"] = True, True
                else:
                    f["emit"] = False
        elif kind == "else":
            if f["taken"]:
                f["emit"] = False
            else:
                if f["kept"]:
                    out.append(ln)
                f["emit"], f["taken"] = True, True
        elif kind == "endif":
            if f["kept"]:
                out.append(ln)
            stack.pop()
        i += 1
    if stack:
        raise SystemExit("unterminated conditional")
    return out, removed


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("file")
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("-K", action="append", default=[])
    ap.add_argument("-U", action="append", default=[])
    a = ap.parse_args(argv)
    defs, keep = {}, set()
    for d in a.D + a.K:
        n, _, v = d.partition("=")
        defs[n] = v or "1"
    keep = {d.partition("=")[0] for d in a.K}
    undefs = set(a.U)
    text = open(a.file).read().split("\n")
    out, removed = process(text, defs, keep, undefs)
    open(a.file, "w").write("\n".join(out))
    left = sorted({n for n in (set(defs) - keep) | undefs for ln in out if re.search(rf"\b{n}\b", ln)})
    print(f"{a.file}: {removed} conditionals resolved; names left: {left}", file=sys.stderr)


if __name__ == "__main__":
    main()
