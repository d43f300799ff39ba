"""Re-point INTEGRATION.md's `# spectralmc_hip.h:<line>` citations at the header lines that declare each bound
function (run after editing include/spectralmc_hip.h; tests/test_capi_host.py checks them)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
hdr = open(os.path.join(ROOT, "include", "spectralmc_hip.h")).read().split("\n")
path = os.path.join(ROOT, "INTEGRATION.md")
text = open(path).read()


def fix(m: re.Match) -> str:
    name, line = m.group(1), int(m.group(3))
    if f"{name}(" in hdr[line - 1]:
        return m.group(0)
    new = next(k + 1 for k, h in enumerate(hdr) if re.search(rf"\b{name}\(", h))
    return m.group(0)[:m.start(3) - m.start(0)] + str(new)


out, n = re.subn(r"_lib\.(smc_\w+)\.argtypes([^#]*?)#\s*spectralmc_hip\.h:(\d+)", fix, text, flags=re.S)
open(path, "w").write(out)
print(f"{n} citations checked, {'changed' if out != text else 'unchanged'}")
