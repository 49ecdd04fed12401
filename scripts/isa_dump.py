"""Per-kernel gfx950 ISA of csrc/gvrt_render.hip, for checking that a source edit left the code unchanged:

    python scripts/isa_dump.py OUTDIR [extra hipcc flags...]

Writes OUTDIR/<kernel>.s (addresses and encodings stripped) for every kernel of the render object plus
OUTDIR/resources.txt (VGPR / SGPR / scratch / occupancy per kernel).  `diff -r` two OUTDIRs."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "3dgvrt_lightfield_amd")
LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    out = os.path.abspath(sys.argv[1])
    os.makedirs(out, exist_ok=True)
    co = os.path.join(out, "render.co")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize",
           "-I" + os.path.join(ROOT, "include"), "-munsafe-fp-atomics", "--cuda-device-only", "--no-gpu-bundle-output", "-c",
           os.path.join(PKG, "csrc", "gvrt_render.hip"), "-o", co, "-Rpass-analysis=kernel-resource-usage",
           *sys.argv[2:]]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.stderr.write(r.stderr)
        sys.exit(r.returncode)
    res = [l for l in r.stderr.splitlines() if re.search(r"Function Name|VGPRs:|SGPRs:|ScratchSize|Occupancy", l)]
    open(os.path.join(out, "resources.txt"), "w").write("\n".join(l.split("remark: ")[-1] for l in res) + "\n")
    dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", "--no-leading-addr", co],
                         capture_output=True, text=True, check=True).stdout
    cur, buf = None, []
    def flush():
        if cur:
            name = re.sub(r"[^A-Za-z0-9_]+", "_", cur)[:180]
            open(os.path.join(out, name + ".s"), "w").write("\n".join(buf) + "\n")
    for line in dis.splitlines():
        m = re.match(r"^([0-9a-f]+ )?<(.+)>:$", line)
        if m:
            flush()
            cur, buf = m.group(2), []
            continue
        if cur:
            line = re.sub(r"\s*//.*$", "", line).rstrip()
            line = re.sub(r"<[^>]*\+0x[0-9a-f]+>", "<L>", line)
            if line:
                buf.append(line)
    flush()
    os.remove(co)


if __name__ == "__main__":
    main()
