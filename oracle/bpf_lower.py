"""Lower BPF LLVM IR (emitted by the image's clang 22) to a BPF ELF object.

TEST INFRASTRUCTURE ONLY — part of the reference-oracle build recipe
(oracle/Makefile).  Nothing in the product imports this.

Why: ROCm's clang 22 can emit BPF IR (`-target bpf -emit-llvm`) but ships
without the BPF code generator; the image's system libLLVM-15 has the BPF
backend.  This script parses the IR with libLLVM-15 through its C API
(ctypes) and emits the object.  LLVM-15 cannot read a few newer IR
attributes/flags, so they are removed textually first — they are
optimisation hints (nuw/nsw/disjoint/captures/...) and do not change the
program's semantics.  Lifetime markers are kept (rewritten to the
LLVM-15 two-operand form) because stack-slot colouring needs them to stay
under BPF's 512-byte stack.

Usage: python3 bpf_lower.py in.ll out.o
"""
import ctypes
import re
import sys

LIBLLVM = "/usr/lib/x86_64-linux-gnu/libLLVM-15.so.1"

_REWRITES = [
    (r"captures\([^)]*\)", ""),
    (r"\brange\([^)]*\)", ""),
    (r"\bmemory\([^)]*\)", ""),
    (r"\binitializes\(\([^)]*\)\)", ""),
    (r"getelementptr inbounds nuw", "getelementptr inbounds"),
    (r"getelementptr nuw", "getelementptr"),
    (r"\bnneg\b", ""),
    (r"\bsamesign\b", ""),
    (r"\bor disjoint\b", "or"),
    (r"\btrunc nuw nsw\b|\btrunc nuw\b|\btrunc nsw\b", "trunc"),
    (r"(?m)^!llvm\.ident = .*$", ""),
    (r"(?m)^attributes #(\d+) = \{.*\}$", r"attributes #\1 = { nounwind }"),
    (r"@llvm\.lifetime\.(start|end)\.p0\(ptr ([^)]*)\)",
     r"@llvm.lifetime.\1.p0(i64 -1, ptr \2)"),
    (r"declare void @llvm\.lifetime\.(start|end)\.p0\(i64 -1, ptr[^)]*\)",
     r"declare void @llvm.lifetime.\1.p0(i64 immarg, ptr nocapture)"),
]


def downlevel(text: str) -> str:
    for pat, rep in _REWRITES:
        text = re.sub(pat, rep, text)
    return text


def lower(ll_path: str, obj_path: str) -> None:
    L = ctypes.CDLL(LIBLLVM)
    for fn in ("LLVMInitializeBPFTargetInfo", "LLVMInitializeBPFTarget",
               "LLVMInitializeBPFTargetMC", "LLVMInitializeBPFAsmPrinter"):
        getattr(L, fn)()
    vp = ctypes.c_void_p
    L.LLVMContextCreate.restype = vp
    L.LLVMCreateMemoryBufferWithMemoryRangeCopy.restype = vp
    L.LLVMCreateMemoryBufferWithMemoryRangeCopy.argtypes = [
        ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    L.LLVMParseIRInContext.argtypes = [vp, vp, ctypes.POINTER(vp),
                                       ctypes.POINTER(ctypes.c_char_p)]
    L.LLVMGetTargetFromTriple.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp),
                                          ctypes.POINTER(ctypes.c_char_p)]
    L.LLVMCreateTargetMachine.restype = vp
    L.LLVMCreateTargetMachine.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p,
                                          ctypes.c_char_p, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_int]
    L.LLVMTargetMachineEmitToFile.argtypes = [vp, vp, ctypes.c_char_p,
                                              ctypes.c_int,
                                              ctypes.POINTER(ctypes.c_char_p)]

    src = downlevel(open(ll_path).read()).encode()
    ctx = L.LLVMContextCreate()
    buf = L.LLVMCreateMemoryBufferWithMemoryRangeCopy(src, len(src), b"m")
    mod, err = vp(), ctypes.c_char_p()
    if L.LLVMParseIRInContext(vp(ctx), vp(buf), ctypes.byref(mod),
                              ctypes.byref(err)):
        raise SystemExit("IR parse error: " + err.value.decode()[:2000])
    tgt = vp()
    if L.LLVMGetTargetFromTriple(b"bpf", ctypes.byref(tgt), ctypes.byref(err)):
        raise SystemExit("no BPF target in libLLVM-15")
    # opt level 2 (Default), reloc default, code model default
    tm = L.LLVMCreateTargetMachine(tgt.value, b"bpf", b"probe", b"", 2, 0, 0)
    if L.LLVMTargetMachineEmitToFile(vp(tm), mod.value, obj_path.encode(), 1,
                                     ctypes.byref(err)):
        raise SystemExit("emit error: " + str(err.value))


if __name__ == "__main__":
    lower(sys.argv[1], sys.argv[2])
