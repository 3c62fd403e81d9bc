"""Split a ThreadSanitizer log of tests/c_harness/dfm_threads_tsan into the
reports that concern libdfm's own host code and those inside the ROCm
runtime.  A report is libdfm's when BOTH racing accesses happen in libdfm or
the harness (their first non-interceptor frame is there): the HIP / HSA
runtimes are not instrumented, so TSan cannot see their internal
synchronisation (worker threads freeing or reusing memory the caller's
thread touched earlier) and flags those as races.
usage: python tools/tsan_filter.py tsan.txt"""
import re
import sys

INTERCEPT = ("malloc", "free", "calloc", "realloc", "memcpy", "memset", "memmove", "operator new", "operator delete",
             "posix_memalign", "__interceptor")


def first_frame(block):
    """The first frame below the sanitizer's interceptors (compiler-rt
    sources, libstdc++'s operator new / delete)."""
    for m in re.finditer(r"#\d+ (.*?) (\S+) \((\S+?)\+", block):
        func, loc, obj = m.groups()
        if "compiler-rt" in loc or "libstdc++" in obj or any(func.startswith(x) for x in INTERCEPT):
            continue
        return func, loc, obj
    return None


def ours(fr):
    return fr is not None and ("libdfm.so" in fr[2] or "dfm_threads" in fr[2])


def main():
    txt = open(sys.argv[1]).read()
    reps = txt.split("WARNING: ThreadSanitizer")[1:]
    own, runtime = [], 0
    for r in reps:
        parts = re.split(r"\n  (?=(?:Previous )?(?:[Ww]rite|[Rr]ead|[Aa]tomic))", r)
        acc = [p for p in parts[1:] if re.match(r"(Previous )?([Ww]rite|[Rr]ead|[Aa]tomic)", p)]
        frs = [first_frame(a.split("\n\n")[0]) for a in acc[:2]]
        if len(frs) == 2 and all(ours(f) for f in frs):
            own.append((r.splitlines()[0].strip(), frs))
        else:
            runtime += 1
    print(f"reports: {len(reps)}; in libdfm / harness code on both sides: {len(own)}; involving the "
          f"uninstrumented ROCm runtime: {runtime}")
    for head, frs in own[:20]:
        print(" ", head, "|", frs[0][0], frs[0][1], "<->", frs[1][0], frs[1][1])
    return 1 if own else 0


if __name__ == "__main__":
    sys.exit(main())
