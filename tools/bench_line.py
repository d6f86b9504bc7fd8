"""One-line summary of a bench.py JSON line (tools/gpu_run.sh prints it after each bench step)."""
import json
import sys


def main(path: str) -> None:
    try:
        d = json.loads(open(path).read().strip().splitlines()[-1])
    except Exception as e:  # a failed run leaves no JSON line
        print(f"{path}: no bench line ({e})")
        return
    r = d.get("roofline") or {}
    b = d.get("bounce") or {}
    s = d.get("sustained") or {}
    p = d.get("parity") or {}
    print(f"{path}: value {d['value']} Mrays/s, {d['ms_per_step']} ms/step, sustained {s.get('value')}, "
          f"kernel {r.get('kernel_ms')} (serial {r.get('kernel_ms_serial')}), host issue/step "
          f"{r.get('host_issue_ms_per_step')}, cull off {d.get('value_cull_off')}, bounce {b.get('value')} "
          f"({b.get('ms_per_step')} ms, mode {str(b.get('compaction_mode'))[:12]}, others {json.dumps(b.get('other_modes'))}), parity {p.get('mismatches')} "
          f"/ {p.get('pixels')}, issue: {d['config'].get('issue', '')[:40]}")


if __name__ == "__main__":
    for p in sys.argv[1:]:
        main(p)
