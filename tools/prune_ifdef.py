#!/usr/bin/env python3
"""Resolve #if / #ifdef / #ifndef blocks that depend only on the given
macros (settled A/B switches), keeping the branch their fixed value selects;
every other conditional is left as it is.  Also drops the switches'
`#ifndef X / #define X v / #endif` default blocks.

  tools/prune_ifdef.py FILE NAME=VALUE [NAME=VALUE ...]   (VALUE: int, or 'undef')
"""
import re
import sys


def main():
    path = sys.argv[1]
    vals = {}
    for kv in sys.argv[2:]:
        k, v = kv.split("=")
        vals[k] = None if v == "undef" else int(v)
    lines = open(path).read().split("\n")

    def evaluate(cond):
        """True/False when cond only involves the macros in vals, else None."""
        names = set(re.findall(r"[A-Za-z_]\w*", cond)) - {"defined"}
        if not names or not names <= set(vals):
            return None
        expr = cond
        expr = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: "1" if vals[m.group(1)] is not None else "0", expr)
        expr = re.sub(r"defined\s+(\w+)", lambda m: "1" if vals[m.group(1)] is not None else "0", expr)
        expr = re.sub(r"\b([A-Za-z_]\w*)\b", lambda m: str(vals[m.group(1)] or 0), expr)
        expr = expr.replace("&&", " and ").replace("||", " or ").replace("!", " not ").replace(" not =", "!=")
        return bool(eval(expr))

    out = []
    # stack entries: (kind, keep_current) kind 'resolved' or 'kept'
    stack = []

    def emitting():
        return all(e[1] for e in stack if e[0] == "resolved")

    i = 0
    while i < len(lines):
        ln = lines[i]
        s = ln.strip()
        m = re.match(r"#\s*(if|ifdef|ifndef|elif|else|endif)\b(.*)", s)
        if m:
            d, rest = m.group(1), m.group(2).split("//")[0].strip()
            if d in ("if", "ifdef", "ifndef"):
                if d == "ifdef":
                    cond = f"defined({rest})"
                elif d == "ifndef":
                    cond = f"!defined({rest})"
                else:
                    cond = rest
                # the default block of a settled switch: #ifndef X / #define X v / #endif
                if d == "ifndef" and rest in vals and i + 2 < len(lines) and \
                        re.match(rf"#\s*define\s+{rest}\b", lines[i + 1].strip()) and lines[i + 2].strip().startswith("#endif"):
                    i += 3
                    continue
                r = evaluate(cond)
                if r is None:
                    stack.append(["kept", True])
                    if emitting():
                        out.append(ln)
                else:
                    stack.append(["resolved", r, r])  # third: some branch taken
                i += 1
                continue
            if d in ("else", "elif"):
                top = stack[-1]
                if top[0] == "kept":
                    if all(e[1] for e in stack[:-1] if e[0] == "resolved"):
                        out.append(ln)
                else:
                    if d == "else":
                        top[1] = not top[2]
                        top[2] = True
                    else:
                        r = evaluate(rest)
                        assert r is not None, f"line {i + 1}: #elif on an unresolved condition"
                        top[1] = (not top[2]) and r
                        top[2] = top[2] or r
                i += 1
                continue
            if d == "endif":
                top = stack.pop()
                if top[0] == "kept" and emitting():
                    out.append(ln)
                i += 1
                continue
        if emitting():
            out.append(ln)
        i += 1
    assert not stack, "unbalanced conditionals"
    open(path, "w").write("\n".join(out))


if __name__ == "__main__":
    main()
