"""Post-mortem of an x86-64 ELF core file without a debugger.

    python tools/probe/core_report.py CORE [--threads N] [--scan BYTES]

Prints, for the thread that took the fatal signal (the first NT_PRSTATUS
note) and for up to N others: its signal, rip/rsp, and the return-address
candidates found by scanning its stack (values that point into executable
file mappings, as file+offset).  The offsets are symbolized on the CPU side
with llvm-symbolizer against the same libraries.  Written for the round-4
namespace-compiler crash, where the process died of SIGSEGV without any
signal handler running."""
import argparse
import os
import struct

NT_PRSTATUS, NT_SIGINFO, NT_FILE = 1, 0x53494749, 0x46494C45
# struct elf_prstatus (x86-64): si_signo..pr_fpvalid; regs at offset 112
REGS = ["r15", "r14", "r13", "r12", "rbp", "rbx", "r11", "r10", "r9", "r8", "rax", "rcx", "rdx", "rsi", "rdi",
        "orig_rax", "rip", "cs", "eflags", "rsp", "ss", "fs_base", "gs_base", "ds", "es", "fs", "gs"]


def notes(f, off, size):
    f.seek(off)
    data = f.read(size)
    i = 0
    while i + 12 <= len(data):
        namesz, descsz, typ = struct.unpack_from("<III", data, i)
        i += 12
        i += (namesz + 3) & ~3
        desc = data[i:i + descsz]
        i += (descsz + 3) & ~3
        yield typ, desc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("core")
    ap.add_argument("--threads", type=int, default=64)
    ap.add_argument("--scan", type=int, default=1 << 16)
    a = ap.parse_args()
    with open(a.core, "rb") as f:
        eh = f.read(64)
        assert eh[:4] == b"\x7fELF" and eh[4] == 2, "not an ELF64 core"
        phoff, = struct.unpack_from("<Q", eh, 32)
        phentsize, phnum = struct.unpack_from("<HH", eh, 54)
        loads, threads, files, siginfo = [], [], [], None
        for k in range(phnum):
            f.seek(phoff + k * phentsize)
            p_type, p_flags, p_offset, p_vaddr, _, p_filesz, p_memsz, _ = struct.unpack("<IIQQQQQQ", f.read(56))
            if p_type == 1:
                loads.append((p_vaddr, p_memsz, p_offset, p_filesz, p_flags))
            elif p_type == 4:
                for typ, desc in notes(f, p_offset, p_filesz):
                    if typ == NT_PRSTATUS:
                        sig, = struct.unpack_from("<i", desc, 12)
                        pid, = struct.unpack_from("<i", desc, 32)
                        regs = dict(zip(REGS, struct.unpack_from("<27Q", desc, 112)))
                        threads.append((pid, sig, regs))
                    elif typ == NT_SIGINFO and siginfo is None:
                        signo, errno_, code = struct.unpack_from("<iii", desc, 0)
                        addr, = struct.unpack_from("<Q", desc, 16)
                        siginfo = (signo, code, addr)
                    elif typ == NT_FILE:
                        count, page = struct.unpack_from("<QQ", desc, 0)
                        ents = [struct.unpack_from("<QQQ", desc, 16 + 24 * j) for j in range(count)]
                        names = desc[16 + 24 * count:].split(b"\0")
                        for (s, e, pg), nm in zip(ents, names):
                            files.append((s, e, pg * page, nm.decode(errors="replace")))

        def where(v):
            for s, e, off, nm in files:
                if s <= v < e:
                    return nm, v - s + off
            return None

        def exec_file(v):
            w = where(v)
            if not w:
                return None
            for vaddr, memsz, _, _, flags in loads:
                if vaddr <= v < vaddr + memsz:
                    return w if flags & 1 else None
            return w  # text segments are often not dumped: assume the file mapping is code

        def read(v, n):
            for vaddr, memsz, off, filesz, _ in loads:
                if vaddr <= v and v + n <= vaddr + filesz:
                    f.seek(off + v - vaddr)
                    return f.read(n)
            return None

        print(f"core {a.core}: {len(threads)} threads, {len(files)} file mappings, siginfo {siginfo and (siginfo[0], siginfo[1], hex(siginfo[2]))}")
        for n, (pid, sig, r) in enumerate(threads[:a.threads]):
            w = where(r["rip"])
            print(f"--- thread {pid} signal {sig} rip {r['rip']:#x} {w and (os.path.basename(w[0]), hex(w[1]))} "
                  f"rsp {r['rsp']:#x} fs_base {r['fs_base']:#x}")
            if n and sig == 0 and n >= 8:
                continue
            stack = read(r["rsp"], a.scan) or read(r["rsp"], 4096)
            if not stack:
                print("    stack not in core")
                continue
            found = 0
            for i in range(0, len(stack) - 7, 8):
                v, = struct.unpack_from("<Q", stack, i)
                w = exec_file(v)
                if w and not w[0].endswith((".dat", ".bin")):
                    print(f"    [rsp+{i:#x}] {os.path.basename(w[0])} +{w[1]:#x}")
                    found += 1
                    if found >= 40:
                        break


if __name__ == "__main__":
    main()
