"""Minimal unifdef: resolve the #if/#ifdef/#ifndef/#else/#endif blocks that test only the given
macros (their values fixed), drop their #define / #ifndef-default lines, keep every other
directive. Used to take rejected build variants out of a kernel source.
  python tools/unifdef.py FILE OD_PAIRS=0 OD_MFMA=0 OCT_PROFILE=undef ...
"""
import re
import sys


def main(path, defs):
    vals = {}
    for d in defs:
        k, v = d.split("=")
        vals[k] = None if v == "undef" else int(v)
    lines = open(path).read().split("\n")
    out = []
    stack = []  # entries: (kind, keep this branch, some branch taken); kind 'ours' / 'other'

    def active():
        return all(k for kind, k, _ in stack if kind == "ours")

    def ev(expr):
        names = set(re.findall(r"[A-Za-z_]\w*", expr)) - {"defined"}
        if not names or not names <= set(vals):
            return None
        e = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: "1" if vals[m.group(1)] is not None else "0", expr)
        e = re.sub(r"defined\s+(\w+)", lambda m: "1" if vals[m.group(1)] is not None else "0", e)
        e = e.replace("&&", " and ").replace("||", " or ")
        e = re.sub(r"!(?!=)", " not ", e)
        e = re.sub(r"[A-Za-z_]\w*", lambda m: m.group(0) if m.group(0) in ("and", "or", "not") else str(vals[m.group(0)] or 0), e)
        return bool(eval(e))

    i = 0
    while i < len(lines):
        ln = lines[i]
        s = ln.strip()
        m = re.match(r"#\s*(ifdef|ifndef|if|else|endif|elif|define)\b\s*(.*)", s)
        if m:
            d, rest = m.group(1), m.group(2).split("//")[0].strip()
            if d in ("ifdef", "ifndef"):
                name = rest.split()[0]
                if name in vals:
                    isdef = vals[name] is not None
                    # "#ifndef X / #define X v / #endif" default blocks vanish
                    k = isdef if d == "ifdef" else not isdef
                    stack.append(("ours", k, k))
                    i += 1
                    continue
                stack.append(("other", True, True))
            elif d == "if":
                r = ev(rest)
                if r is not None:
                    stack.append(("ours", r, r))
                    i += 1
                    continue
                stack.append(("other", True, True))
            elif d == "elif":
                if stack and stack[-1][0] == "ours":
                    _, _, taken = stack.pop()
                    r = ev(rest)
                    if r is None:
                        raise SystemExit(f"{path}:{i + 1}: unresolvable #elif in a resolved block")
                    k = (not taken) and r
                    stack.append(("ours", k, taken or k))
                    i += 1
                    continue
            elif d == "else":
                if stack[-1][0] == "ours":
                    kind, _, taken = stack.pop()
                    stack.append((kind, not taken, True))
                    i += 1
                    continue
            elif d == "endif":
                kind, _, _ = stack.pop()
                if kind == "ours":
                    i += 1
                    continue
            elif d == "define":
                name = rest.split()[0].split("(")[0]
                if name in vals:
                    i += 1
                    continue
        if active():
            out.append(ln)
        i += 1
    assert not stack, stack
    open(path, "w").write("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
