"""Resolve preprocessor conditionals on a set of macros (a small unifdef for pruning A/B variants).

    python tools/unifdef.py FILE -UMACRO ... [-DMACRO ...]

Every #if / #ifdef / #ifndef / #elif whose condition mentions only listed macros (through
defined(X), #ifdef X, #ifndef X, &&, ||, !, parentheses) is evaluated and the dead branch removed;
conditionals on other macros are kept verbatim. The file is rewritten in place.
"""
import re
import sys


def cond_expr(line):
    s = line.strip()
    if s.startswith("#ifdef"):
        return "defined(%s)" % s.split()[1]
    if s.startswith("#ifndef"):
        return "!defined(%s)" % s.split()[1]
    if s.startswith("#elif"):
        return s[len("#elif"):].split("//")[0].strip()
    return s[len("#if"):].split("//")[0].strip()


def evaluate(expr, undef, define):
    names = set(re.findall(r"defined\s*\(\s*(\w+)\s*\)", expr))
    rest = re.sub(r"defined\s*\(\s*\w+\s*\)", "", expr)
    if re.search(r"[A-Za-z_]\w*", rest) or not names or not names <= (undef | define):
        return None
    py = re.sub(r"defined\s*\(\s*(\w+)\s*\)", lambda m: "True" if m.group(1) in define else "False", expr)
    py = py.replace("&&", " and ").replace("||", " or ")
    py = re.sub(r"!(?!=)", " not ", py)
    return bool(eval(py))


def main():
    path = sys.argv[1]
    undef = {a[2:] for a in sys.argv[2:] if a.startswith("-U")}
    define = {a[2:] for a in sys.argv[2:] if a.startswith("-D")}
    out = []
    # stack of frames: (resolved, taken_any, emitting_now, parent_emitting)
    stack = []
    emitting = True
    for line in open(path).read().split("\n"):
        s = line.strip()
        if s.startswith(("#if ", "#ifdef", "#ifndef", "#if(")):
            v = evaluate(cond_expr(s), undef, define)
            if v is None:
                stack.append([False, False, emitting, emitting])
                if emitting:
                    out.append(line)
            else:
                stack.append([True, v, emitting and v, emitting])
                emitting = emitting and v
            continue
        if s.startswith("#elif") and stack:
            fr = stack[-1]
            if not fr[0]:
                if fr[3]:
                    out.append(line)
                continue
            v = evaluate(cond_expr(s), undef, define)
            if v is None:
                raise SystemExit("%s: unresolvable #elif inside a resolved chain: %s" % (path, s))
            take = v and not fr[1]
            fr[1] = fr[1] or v
            emitting = fr[3] and take
            continue
        if s.startswith("#else") and stack:
            fr = stack[-1]
            if not fr[0]:
                if fr[3]:
                    out.append(line)
                continue
            emitting = fr[3] and not fr[1]
            fr[1] = True
            continue
        if s.startswith("#endif") and stack:
            fr = stack.pop()
            emitting = fr[3]
            if not fr[0] and emitting:
                out.append(line)
            continue
        if emitting:
            out.append(line)
    open(path, "w").write("\n".join(out))


if __name__ == "__main__":
    main()
