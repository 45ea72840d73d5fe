"""The product kernels carry no instruction-emitting inline asm.

LLVM's hazard recognizer does not see an inline-asm statement as a reader of the registers it
uses, so gfx950's 3-wait-state rule after a v_dot* write was violated once the max-ilp scheduler
moved an asm multiply-add right behind the dot4 that produced its operand (DESIGN.md section 3,
tools/asm_hazards.py).  Empty asm statements (register-placement barriers, which emit nothing and
which the recognizer counts as 0 wait states) are the only asm left."""
import os
import re

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ggrs_amd", "csrc")
_ASM = re.compile(r"\basm\s*(?:volatile\s*)?\(\s*\"([^\"]*)\"")


def test_no_instruction_emitting_inline_asm():
    found = []
    for name in sorted(os.listdir(CSRC)):
        if not name.endswith((".h", ".hip", ".cpp")):
            continue
        text = open(os.path.join(CSRC, name)).read()
        for m in _ASM.finditer(text):
            if m.group(1).strip():
                line = text.count("\n", 0, m.start()) + 1
                found.append(f"{name}:{line}: {m.group(1)}")
    assert not found, found


def test_hazard_checker_flags_the_round4_pattern():
    """tools/asm_hazards.py on the instruction sequence hipcc -S produced for particles.hip at
    9732acd^ under max-ilp (the two dot4 chains ending, then the asm reading the accumulator)."""
    import importlib.util
    root = os.path.dirname(CSRC.rstrip("/").rsplit("/", 1)[0])
    spec = importlib.util.spec_from_file_location("asm_hazards", os.path.join(root, "tools", "asm_hazards.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    bad = """
	v_dot4_u32_u8 v27, v26, s85, v27
	v_dot4_u32_u8 v30, v26, s84, v30
	;;#ASMSTART
	v_mad_u32_u24 v32, v59, v27, v84
	;;#ASMEND
	s_nop 1
	v_mul_hi_u32_u24_e32 v31, 0x808081, v27
""".splitlines()
    blocks, hazards = mod.scan(bad)
    assert len(blocks) == 1 and len(hazards) == 1 and hazards[0][2] == 27 and hazards[0][4] == 1
    good = """
	v_dot4_u32_u8 v27, v26, s85, v27
	v_dot4_u32_u8 v30, v26, s84, v30
	s_nop 1
	;;#ASMSTART
	v_mad_u32_u24 v32, v59, v27, v84
	;;#ASMEND
""".splitlines()
    assert mod.scan(good)[1] == []
