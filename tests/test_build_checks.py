"""The build's code-object checks (CPU): the store-data hazard scan (build.scan_store_hazards, DESIGN.md section 3
"128-bit stores") and the wait-state scan of the classes the compiler does not pad around inline assembly
(build.scan_valu_hazards: DPP, readlane, SGPR -> VMEM, lane select, transcendental forwarding) on disassembly
snippets shaped like llvm-objdump's, and both checks running over the product's fused-kernel objects when they are
present."""
import json
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "differentiable-tube-mpc_amd"))

import build  # noqa: E402

HEAD = "\n<_ZN5dtmpc2fk16tube_fast_kernelILi5ELi4ELi2EEEvNS0_2FKE>:\n"


def _scan(body):
    return build.scan_store_hazards(HEAD + "".join(f"\t{line}\n" for line in body))


def test_hazard_found_when_data_register_written_next():
    h = _scan(["buffer_store_dwordx4 v[14:17], v218, s[52:55], s91 offen", "v_mov_b32_e32 v15, v67",
               "s_endpgm"])
    assert len(h) == 1 and "v15" in h[0][2] and "tube_fast_kernel" in h[0][0]


def test_hazard_found_one_instruction_later():
    h = _scan(["buffer_store_dwordx4 v[14:17], v218, s[52:55], s91 offen", "v_add_f32_e32 v3, v4, v5",
               "v_pk_add_f32 v[16:17], v[20:21], v[22:23]"])
    assert len(h) == 1


def test_no_hazard_after_two_wait_states():
    assert not _scan(["buffer_store_dwordx4 v[14:17], v218, s[52:55], s91 offen", "s_nop 1",
                      "v_mov_b32_e32 v14, v211"])
    assert not _scan(["buffer_store_dwordx4 v[14:17], v218, s[52:55], s91 offen", "v_add_f32_e32 v3, v4, v5",
                      "v_add_f32_e32 v6, v4, v5", "v_mov_b32_e32 v14, v211"])


def test_no_hazard_for_other_registers_or_narrow_stores():
    assert not _scan(["buffer_store_dwordx4 v[14:17], v218, s[52:55], s91 offen", "v_mov_b32_e32 v18, v211"])
    assert not _scan(["buffer_store_dwordx2 v[14:15], v218, s[52:55], s91 offen", "v_mov_b32_e32 v14, v211"])


def test_product_objects_have_no_hazard():
    path = os.path.join(REPO, "differentiable-tube-mpc_amd", "build", "obj", "store_hazards.json")
    if not os.path.exists(path):
        pytest.skip("no product build in this tree (build.py writes build/obj/store_hazards.json)")
    rep = json.load(open(path))
    assert rep and all(len(v) == 0 for v in rep.values()), {k: len(v) for k, v in rep.items()}


def _vscan(body):
    return build.scan_valu_hazards(HEAD + "".join(f"\t{line}  // 000000001234: 00000000\n" for line in body))


@pytest.mark.parametrize("body,cls", [
    (["v_fma_f64 v[92:93], v[14:15], v[92:93], v[18:19]",
      "v_mov_b32_dpp v4, v92 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"], "VALU->DPP"),
    (["v_add_f32_e32 v7, v4, v5", "s_nop 0", "v_mov_b32_dpp v4, v7 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf"],
     "VALU->DPP"),
    (["v_add_f32_e32 v7, v4, v5", "v_readfirstlane_b32 s4, v7"], "VALU->READLANE"),
    (["v_readfirstlane_b32 s0, v3", "s_nop 1", "buffer_load_dwordx4 v[10:13], v20, s[84:87], s0 offen"],
     "VALU_SGPR->VMEM"),
    (["v_readfirstlane_b32 s5, v3", "v_readlane_b32 s6, v9, s5"], "VALU_SGPR->LANESEL"),
    (["v_exp_f32_e32 v3, v2", "v_add_f32_e32 v4, v3, v5"], "TRANS->VALU"),
])
def test_valu_hazard_classes_found(body, cls):
    h = _vscan(body)
    assert [x[0] for x in h] == [cls], h


@pytest.mark.parametrize("body", [
    ["v_fma_f64 v[92:93], v[14:15], v[92:93], v[18:19]", "s_nop 1",
     "v_mov_b32_dpp v4, v92 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"],
    ["v_add_f32_e32 v7, v4, v5", "v_mov_b32_dpp v4, v8 quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf"],
    ["v_add_f32_e32 v7, v4, v5", "s_nop 0", "v_readfirstlane_b32 s4, v7"],
    ["v_readfirstlane_b32 s0, v3", "s_nop 4", "buffer_load_dwordx4 v[10:13], v20, s[84:87], s0 offen"],
    ["v_exp_f32_e32 v3, v2", "s_nop 0", "v_add_f32_e32 v4, v3, v5"],
    ["v_exp_f32_e32 v3, v2", "v_log_f32_e32 v4, v3"],
])
def test_valu_hazard_classes_clear(body):
    assert not _vscan(body)


def test_product_objects_have_no_wait_state_hazard():
    path = os.path.join(REPO, "differentiable-tube-mpc_amd", "build", "obj", "valu_hazards.json")
    if not os.path.exists(path):
        pytest.skip("no product build with the wait-state scan in this tree (build.py writes build/obj/valu_hazards.json)")
    rep = json.load(open(path))
    assert rep and all(len(v) == 0 for v in rep.values()), {k: len(v) for k, v in rep.items()}


def _fscan(body):
    """scan_flow_copies on instructions at consecutive 4-byte offsets; "-> N" marks a branch to instruction N."""
    lines = []
    for n, ins in enumerate(body):
        tgt = ""
        if " -> " in ins:
            ins, to = ins.split(" -> ")
            tgt = f" <_ZN5dtmpc4fk6416tube_fast_kernelILi5ELi2ELi2EEEvNS0_2FKE+0x{4 * int(to):x}>"
        lines.append(f"\t{ins}  // {0x1000 + 4 * n:012X}: 00000000{tgt}\n")
    return build.scan_flow_copies("\n<_ZN5dtmpc4fk6416tube_fast_kernelILi5ELi2ELi2EEEvNS0_2FKE>:\n" + "".join(lines))


# the round-6 finding (profiles/r06/flow_copy_root_cause.txt): a live-range-split copy at the head of an if / else flow
# block runs with the then-lanes' exec mask only
FLOW_BAD = ["v_cmp_le_f64_e32 vcc, s[68:69], v[28:29]", "s_and_saveexec_b64 s[0:1], vcc", "s_xor_b64 s[0:1], exec, s[0:1]",
            "s_cbranch_execz 3 -> 6", "v_mul_f64 v[28:29], v[28:29], v[28:29]", "v_div_fixup_f64 v[126:127], v[34:35], v[28:29], -1.0",
            "v_accvgpr_write_b32 a10, v98", "v_accvgpr_write_b32 a11, v99", "s_andn2_saveexec_b64 s[0:1], s[0:1]",
            "s_cbranch_execz 2 -> 11", "v_add_f64 v[126:127], v[20:21], -s[28:29]", "s_or_b64 exec, exec, s[0:1]",
            "s_endpgm"]


def test_flow_block_copy_found():
    h = _fscan(FLOW_BAD)
    assert [x[2] for x in h] == ["v_accvgpr_write_b32 a10, v98", "v_accvgpr_write_b32 a11, v99"]


def test_flow_block_clear_without_copies_or_for_lane_writes():
    # the same if / else with the copies before the branch (full exec): nothing at the flow block's head
    good = (FLOW_BAD[:1] + ["v_accvgpr_write_b32 a10, v98", "v_accvgpr_write_b32 a11, v99"] + FLOW_BAD[1:3] +
            ["s_cbranch_execz 3 -> 8"] + FLOW_BAD[4:6] + FLOW_BAD[8:9] + ["s_cbranch_execz 2 -> 11"] + FLOW_BAD[10:])
    assert not _fscan(good)
    # SGPR spills by v_writelane ignore exec: not a partial write
    lane = FLOW_BAD[:6] + ["v_writelane_b32 v253, s30, 8", "v_writelane_b32 v253, s31, 9"] + FLOW_BAD[8:]
    assert not _fscan(lane)


def test_product_objects_have_no_flow_block_copy():
    path = os.path.join(REPO, "differentiable-tube-mpc_amd", "build", "obj", "flow_copies.json")
    if not os.path.exists(path):
        pytest.skip("no product build with the flow-block scan in this tree (build.py writes build/obj/flow_copies.json)")
    rep = json.load(open(path))
    assert rep and all(len(v) == 0 for v in rep.values()), {k: len(v) for k, v in rep.items() if v}


def test_unit_flags_and_checked_units_are_built_units():
    """UNIT_FLAGS (the iterative-ILP units, DESIGN.md section 3 "The one-lane kernels' instruction schedule") and the
    f64 resource check name translation units the build compiles: a renamed unit must not silently lose its flags or
    its scratch check."""
    units = {os.path.splitext(os.path.basename(s))[0] for s in build.SRCS}
    assert set(build.UNIT_FLAGS) <= units, set(build.UNIT_FLAGS) - units
    assert set(build.RESOURCE_CHECKED) <= units, set(build.RESOURCE_CHECKED) - units
    assert {"dtmpc_fast_ilp", "dtmpc_fast64_ilp"} <= set(build.UNIT_FLAGS)
    assert "dtmpc_fast64_ilp" in build.RESOURCE_CHECKED


def test_object_key_follows_the_source(tmp_path):
    """build._key covers the source text: the check that refuses an object whose sources changed while hipcc ran
    (device and host passes read the file minutes apart) compares the key before and after the compile."""
    src = tmp_path / "x.hip"
    src.write_text("int a;\n")
    k0 = build._key(["hipcc", "-c"], str(src))
    src.write_text("int b;\n")
    assert build._key(["hipcc", "-c"], str(src)) != k0
