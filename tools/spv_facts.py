"""Parse-only reader of the reference's compiled fragment shader (res/shaders/volume_frag.spv).

TEST INFRASTRUCTURE. The SPIR-V module is read as data: words are decoded, nothing is
executed or compiled. It pins, from the artifact the reference actually loads at run time
(`/root/reference/src/rendering/offscreen_pass.cpp:618-619`), the facts the oracle relies on:

* the loop constants 1.8 (ray_dist) and 0.005 (step_size) of `volume.frag:29-30`;
* that no result carries `NoContraction` (42) or `RelaxedPrecision` (0): the driver may
  contract `ray_pos += ray_dir * step_size` (`volume.frag:47`) and the composite
  (`:44-45`) into FMAs, and must evaluate them at full float32 precision;
* the composite's operand order: `(sample.rgb * sample.a) * color.a` as two
  `OpVectorTimesScalar`, then `OpFAdd`; `color.a * (1 - sample.a)`;
* the ray advance: `OpVectorTimesScalar(ray_dir, step_size)` then `OpFAdd(ray_pos, ·)`;
* the normalisation `(density - min) / (max - min)` as `OpFSub`, `OpFSub`, `OpFDiv`;
* the loop bound `int(ray_dist / step_size)` as `OpFDiv` + `OpConvertFToS`;
* two `OpImageSampleImplicitLod` (3D volume, 1D TF) and no explicit `Fma` ext-inst.

Usage: python tools/spv_facts.py [path.spv] [--json out.json]  (prints the facts as JSON).
The SPIR-V format is the Khronos "SPIR-V Specification" (Unified), sections 2.3 (physical
layout) and 3 (binary form: opcodes and decoration numbers cited below).
"""
import json
import struct
import sys

MAGIC = 0x07230203

# SPIR-V opcodes used here (SPIR-V spec §3.52 "Instructions")
OP = {
    5: "OpName", 6: "OpMemberName", 11: "OpExtInstImport", 12: "OpExtInst",
    15: "OpEntryPoint", 16: "OpExecutionMode",
    19: "OpTypeVoid", 20: "OpTypeBool", 21: "OpTypeInt", 22: "OpTypeFloat",
    23: "OpTypeVector", 24: "OpTypeMatrix", 25: "OpTypeImage", 27: "OpTypeSampledImage",
    30: "OpTypeStruct", 32: "OpTypePointer", 33: "OpTypeFunction",
    41: "OpConstantTrue", 42: "OpConstantFalse", 43: "OpConstant",
    44: "OpConstantComposite", 54: "OpFunction", 56: "OpFunctionEnd", 59: "OpVariable",
    61: "OpLoad", 62: "OpStore", 65: "OpAccessChain", 71: "OpDecorate",
    72: "OpMemberDecorate", 79: "OpVectorShuffle", 80: "OpCompositeConstruct",
    81: "OpCompositeExtract", 82: "OpCompositeInsert",
    87: "OpImageSampleImplicitLod", 88: "OpImageSampleExplicitLod",
    110: "OpConvertFToS", 111: "OpConvertSToF",
    129: "OpFAdd", 131: "OpFSub", 133: "OpFMul", 136: "OpFDiv", 142: "OpVectorTimesScalar",
    154: "OpAny", 155: "OpAll", 166: "OpLogicalOr", 167: "OpLogicalAnd",
    177: "OpSLessThan", 184: "OpFOrdLessThan", 186: "OpFOrdGreaterThan",
    245: "OpPhi", 246: "OpLoopMerge", 247: "OpSelectionMerge", 248: "OpLabel",
    249: "OpBranch", 250: "OpBranchConditional", 253: "OpReturn",
}
DECORATION_RELAXED_PRECISION = 0   # SPIR-V spec §3.20 "Decoration"
DECORATION_NO_CONTRACTION = 42
GLSL_STD_450_FMA = 50              # GLSL.std.450 extended instruction "Fma"


def parse(data: bytes):
    """Return (header, [(opcode, [operand words])]) of a little-endian SPIR-V module."""
    if len(data) % 4 or len(data) < 20:
        raise ValueError("not a SPIR-V module (size)")
    words = struct.unpack("<%dI" % (len(data) // 4), data)
    if words[0] != MAGIC:
        raise ValueError("not a little-endian SPIR-V module (magic %#x)" % words[0])
    header = {"version": words[1], "generator": words[2], "bound": words[3]}
    insts, i = [], 5
    while i < len(words):
        wc, op = words[i] >> 16, words[i] & 0xFFFF
        if wc == 0 or i + wc > len(words):
            raise ValueError("truncated instruction at word %d" % i)
        insts.append((op, list(words[i + 1:i + wc])))
        i += wc
    return header, insts


def _string(ops):
    b = struct.pack("<%dI" % len(ops), *ops)
    return b.split(b"\0", 1)[0].decode("utf-8", "replace")


def facts(data: bytes) -> dict:
    header, insts = parse(data)
    names, float_types, consts, decorations, ext_sets = {}, set(), {}, [], {}
    int_consts, chains = {}, {}
    defs = {}    # result id -> (opname, operand ids after (type, result))
    body = []    # function-body arithmetic in program order
    int_types = set()
    for op, ops in insts:
        name = OP.get(op, "Op%d" % op)
        if op == 21:
            int_types.add(ops[0])
        elif op == 43 and ops[0] in int_types:
            int_consts[ops[1]] = ops[2]
        elif op == 65:   # OpAccessChain: base[idx...] (member / component selection)
            chains[ops[1]] = (ops[2], ops[3:])
        if op == 5:
            names[ops[0]] = _string(ops[1:])
        elif op == 22:
            float_types.add(ops[0])
        elif op == 11:
            ext_sets[ops[0]] = _string(ops[1:])
        elif op == 43 and ops[0] in float_types:
            consts[ops[1]] = struct.unpack("<f", struct.pack("<I", ops[2]))[0]
        elif op in (71, 72):
            decorations.append((name, ops))
        if op in (12, 61, 79, 81, 87, 110, 129, 131, 133, 136, 142):
            defs[ops[1]] = (name, ops[2:])
            body.append((name, ops[1], ops[2:]))

    def label(i):
        if i in consts:
            return repr(consts[i])
        if i in names:
            return names[i]
        if i in defs:
            return "%" + str(i)
        return "#" + str(i)

    def pointer(i):
        """A variable or an access chain into one: `color[3]`, `u_ubo[4]`."""
        if i in chains:
            base, idx = chains[i]
            return "%s[%s]" % (pointer(base),
                               ",".join(str(int_consts.get(k, "%" + str(k))) for k in idx))
        return names.get(i, "%" + str(i))

    def expr(i, depth=4):
        """Operator tree of an id, a few levels deep (loads print the variable's name)."""
        if i in consts:
            return repr(consts[i])
        if i not in defs or depth == 0:
            return label(i)
        opn, args = defs[i]
        if opn == "OpLoad":
            return pointer(args[0])
        if opn == "OpCompositeExtract":
            return "%s[%s]" % (expr(args[0], depth - 1), ",".join(str(a) for a in args[1:]))
        if opn == "OpVectorShuffle":
            return "%s.swz(%s)" % (expr(args[0], depth - 1), ",".join(str(a) for a in args[2:]))
        if opn == "OpImageSampleImplicitLod":
            return "texture(%s)" % expr(args[0], depth - 1)
        return "%s(%s)" % (opn[2:], ", ".join(expr(a, depth - 1) for a in args))

    no_contraction = [d for d in decorations
                      if (d[0] == "OpDecorate" and d[1][1] == DECORATION_NO_CONTRACTION) or
                      (d[0] == "OpMemberDecorate" and d[1][2] == DECORATION_NO_CONTRACTION)]
    relaxed = [d for d in decorations
               if (d[0] == "OpDecorate" and d[1][1] == DECORATION_RELAXED_PRECISION) or
               (d[0] == "OpMemberDecorate" and d[1][2] == DECORATION_RELAXED_PRECISION)]
    fma_ext = [b for b in body if b[0] == "OpExtInst" and
               ext_sets.get(b[2][0], "") == "GLSL.std.450" and b[2][1] == GLSL_STD_450_FMA]
    arith = [{"op": b[0][2:], "expr": expr(b[1])} for b in body
             if b[0] in ("OpFAdd", "OpFSub", "OpFMul", "OpFDiv", "OpVectorTimesScalar",
                         "OpConvertFToS")]
    samples = [b for b in body if b[0] == "OpImageSampleImplicitLod"]
    return {
        "header": header,
        "float_constants": sorted(set(round(v, 9) for v in consts.values())),
        "ray_dist_1_8_present": any(v == struct.unpack("<f", struct.pack("<f", 1.8))[0]
                                    for v in consts.values()),
        "step_0_005_present": any(v == struct.unpack("<f", struct.pack("<f", 0.005))[0]
                                  for v in consts.values()),
        "no_contraction_decorations": len(no_contraction),
        "relaxed_precision_decorations": len(relaxed),
        "explicit_fma_ext_insts": len(fma_ext),
        "image_samples": len(samples),
        "names": sorted(set(names.values())),
        "arithmetic": arith,
    }


def main(argv):
    path = "/root/reference/res/shaders/volume_frag.spv"
    out = None
    args = list(argv)
    if "--json" in args:
        k = args.index("--json")
        out = args[k + 1]
        del args[k:k + 2]
    if args:
        path = args[0]
    with open(path, "rb") as f:
        fx = facts(f.read())
    text = json.dumps(fx, indent=1)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main(sys.argv[1:])
