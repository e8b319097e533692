"""Generate the wave-flume fixtures (moving boundaries + floating body) by running the
REFERENCE solver (build container only: needs the binaries of ``make -C oracle``).

tests/golden/bi4/flume_<variant>/
  CaseFlume.xml / .bi4 [/ _Normals.nbi4]   case written by genflume_ref: fixed walls, a piston
                                           (mvrectsinu), a flap (wait -> mvrotsinu), a floating
                                           box (RigidAlgorithm=1) and still water
  ref.npz                                  reference run -nsteps:N -svsteps:1 -saveposdouble:1:
                                           PART snapshots (partdump_ref, sorted by idp) at the
                                           kept steps, the PART times, and the floating-body
                                           state of every PART (PartFloat.fbi4 via ftdump_ref:
                                           center, fvel, fomega)
Usage: python tests/golden/make_flume_case.py
"""
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(ROOT, "oracle", "_ref")
sys.path.insert(0, HERE)
from make_golden import load_dump  # noqa: E402

# variant: (dp, step 1 Verlet / 2 Symplectic, ddt, boundary 1 DBC / 2 mDBC, nsteps, kept steps)
VARIANTS = {
    "verlet_ddt2": (0.025, 1, 2, 1, 100, (1, 10, 50, 100)),
    "symplectic_ddt1_mdbc": (0.025, 2, 1, 2, 60, (1, 10, 60)),
    # a fast, wide flap (no wait, 8 Hz, 12 degrees): its mDBC particles cross cell columns
    # within the run (the slab hand-over of turned normals, tests/test_bodies.py)
    "symplectic_ddt1_mdbc_fastflap": (0.025, 2, 1, 2, 80, (1, 40, 80), ("1.2", "0.3", "0.4", "0.2", "0", "8", "12")),
    # the floating box with imposed velocities ("none" components stay free) and external
    # forces (JLinearValue tables of <floating>, FtApplyImposedVel / GetFtExternalForce*)
    "verlet_ddt2_ftvel": (0.025, 1, 2, 1, 100, (1, 10, 50, 100), (), "ftvel"),
    # the same tables in the reference's other forms: <linearvel> from a data file
    # (JLinearValue::LoadFile) and <angularvel> rows out of time order, which JLinearValue walks
    # as they come (FindTime's persistent Position)
    "verlet_ddt2_ftvel_file_unordered": (0.025, 1, 2, 1, 100, (1, 10, 50, 100), (), "ftvelfile"),
    # mDBC on the floating box too (genflume_ref ftnormals=1: UseNormalsFt, the normals turned
    # with the body, JSphCpuSingle.cpp:988-999), Verlet and Symplectic
    "verlet_ddt2_mdbc_ftnor": (0.025, 1, 2, 2, 100, (1, 10, 50, 100),
                               ("1.2", "0.3", "0.4", "0.2", "0.004", "2", "3", "1")),
    "symplectic_ddt1_mdbc_ftnor": (0.025, 2, 1, 2, 60, (1, 10, 60),
                                   ("1.2", "0.3", "0.4", "0.2", "0.004", "2", "3", "1")),
    # MDBCCorrector=1: mDBC also before the Symplectic corrector's interaction (JSph.cpp:639,
    # JSphCpuSingle.cpp:525), with the floating normals
    "symplectic_ddt1_mdbc_corr": (0.025, 2, 1, 2, 60, (1, 10, 60),
                                  ("1.2", "0.3", "0.4", "0.2", "0.004", "2", "3", "1"), "mdbccorr"),
    # other motion programs (JMotion.cpp:556-700, JMotionObj.cpp:368-580): the piston as the
    # child of a virtual object (its own circular movements on top of its parent's sinusoid,
    # its axes moved by the parent), the flap turning at constant speed then accelerating
    "verlet_ddt2_motion_nested_cir": (0.025, 1, 2, 1, 60, (1, 10, 30, 60), (), "motion_nested_cir"),
    "symplectic_ddt1_motion_nested_cir": (0.025, 2, 1, 1, 40, (1, 10, 40), (), "motion_nested_cir"),
    # positions / angles from data files, a flash movement, mvnull, an event with a finish
    "verlet_ddt2_motion_files_flash": (0.025, 1, 2, 1, 60, (1, 10, 30, 60), (), "motion_files_flash"),
    # Symmetry (y = 0 mirror) with ShiftMode NoFixed and moving boundaries (the piston and the
    # flap; no floating box: genflume_ref nofloat=1, the reference refuses Symmetry with
    # floating bodies): the images of a moving p2 join the shifting sums before the first
    # fixed p2 in the reference's order (JSphCpu.cpp:743-750,793-796)
    "verlet_ddt2_sym_nofixed": (0.025, 1, 2, 1, 60, (1, 10, 30, 60),
                                ("1.2", "0.3", "0.4", "0.2", "0.004", "2", "3", "0", "1"), "sym_nofixed"),
    "symplectic_ddt1_sym_nofixed": (0.025, 2, 1, 1, 40, (1, 10, 40),
                                    ("1.2", "0.3", "0.4", "0.2", "0.004", "2", "3", "0", "1"), "sym_nofixed"),
}

# <floating> additions of the XML edits (JCasePartBlock_Floating::ReadXml, JCaseParts.cpp:270-285)
XML_EDITS = {
    "ftvel": ('<linearvel><vel time="0" x="0.05" y="none" z="none"/><vel time="0.006" x="0.2"/>'
              '<vel time="0.02" x="-0.1" z="0.05"/><vel time="0.025" x="0" z="none"/></linearvel>'
              '<angularvel><vel time="0" x="none" y="0.4" z="none"/><vel time="0.012" x="none" y="-0.6" z="none"/>'
              '</angularvel>'
              '<linearforce><force time="0" x="0" y="0.2" z="3"/><force time="0.03" x="0.5" y="0.2" z="1"/>'
              '</linearforce>'
              '<angularforce><force time="0" x="0.002" y="0" z="-0.001"/><force time="0.015" x="0" y="0" z="0.003"/>'
              '</angularforce>'),
    "ftvelfile": ('<linearvel file="FtLinVel.csv"/>'
                  '<angularvel><vel time="0" x="none" y="0.4" z="none"/><vel time="0.02" x="none" y="-0.2" z="none"/>'
                  '<vel time="0.008" x="none" y="-0.6" z="none"/><vel time="0.03" x="none" y="0.1" z="none"/>'
                  '</angularvel>'
                  '<linearforce><force time="0.03" x="0.5" y="0.2" z="1"/><force time="0" x="0" y="0.2" z="3"/>'
                  '</linearforce>'),
    # (anchor, text): the text goes before the anchor
    "mdbccorr": ("</parameters>", '<parameter key="MDBCCorrector" value="1"/>\n'),
    # {"replace": [(old, new)]}: text replaced
    "sym_nofixed": {"replace": [('<parameter key="Shifting" value="0"/>',
                                 '<parameter key="Symmetry" value="1"/>\n<parameter key="Shifting" value="2"/>\n'
                                 '<parameter key="ShiftCoef" value="-2"/>\n<parameter key="ShiftTFS" value="0"/>')]},
    # {"motion": text}: the case's whole <motion> program replaced
    "motion_nested_cir": {"motion": """<motion>
<obj><begin mov="1" start="0"/>
<mvrectsinu id="1" duration="100"><freq x="2" y="0" z="0"/><ampl x="0.01" y="0" z="0"/><phase x="0" y="0" z="0"/></mvrectsinu>
<objreal ref="0"><begin mov="1" start="0.002"/>
<mvcir id="1" duration="0.004" next="2"><axisp1 x="0.05" y="0" z="0.2"/><axisp2 x="0.05" y="1" z="0.2"/><ref x="0.07" y="0" z="0.2"/><vel ang="1500"/></mvcir>
<mvcirace id="2" duration="0.004" next="3"><axisp1 x="0.05" y="0" z="0.2"/><axisp2 x="0.05" y="1" z="0.2"/><ref x="0.07" y="0" z="0.2"/><ace ang="-20000"/></mvcirace>
<mvcirsinu id="3" duration="100"><axisp1 x="0.05" y="0" z="0.2"/><axisp2 x="0.05" y="1" z="0.2"/><ref x="0.07" y="0" z="0.2"/><freq v="5"/><ampl v="8"/></mvcirsinu>
</objreal>
</obj>
<objreal ref="1"><begin mov="1" start="0"/>
<wait id="1" duration="0.003" next="2"/>
<mvrot id="2" duration="0.005" next="3" anglesunits="radians"><axisp1 x="1.2" y="0" z="0"/><axisp2 x="1.2" y="1" z="0"/><vel ang="-0.8"/></mvrot>
<mvrotace id="3" duration="100"><axisp1 x="1.2" y="0" z="0"/><axisp2 x="1.2" y="1" z="0"/><ace ang="500"/></mvrotace>
</objreal>
</motion>"""},
    "motion_files_flash": {"motion": """<motion>
<objreal ref="0"><begin mov="1" start="0"/>
<mvrectfile id="1" duration="0.006" next="2"><file name="PistonPos.csv" fields="4" fieldtime="0" fieldx="1" fieldz="3"/></mvrectfile>
<mvrect id="2" duration="-0.01" next="3"><vel x="0.2" y="0" z="0"/></mvrect>
<mvrotfile id="3" duration="100" anglesunits="radians"><axisp1 x="0.05" y="0" z="0"/><axisp2 x="0.05" y="1" z="0"/><file name="PistonAng.csv"/></mvrotfile>
</objreal>
<objreal ref="1"><begin mov="1" start="0"/><begin mov="2" start="0.004" finish="0.012"/>
<mvnull id="1"/>
<mvfile id="2" duration="100"><file name="FlapPos.csv" fields="3" fieldtime="0" fieldx="1"/></mvfile>
</objreal>
</motion>"""},
}
# data files of the XML edits (written beside the case)
DATA_FILES = {
    "ftvelfile": {"FtLinVel.csv": "# time;vx;vy;vz (m/s)\n0;0.05;none;none\n0.02;-0.1;none;0.05\n"
                                  "0.006;0.2;none;none\n0.025;0;none;none\n"},
    "motion_files_flash": {
        "PistonPos.csv": "# time;x;unused;z\n0;0;9;0\n0.002;0.001;9;0.0005\n0.004;0.0035;9;0.001\n0.01;0.004;9;0\n",
        "PistonAng.csv": "# time ang(rad)\n0 0\n0.004 0.02\n0.02 -0.01\n",
        "FlapPos.csv": "0,0,5\n0.003,-0.002,5\n0.006,-0.001,5\n0.01,-0.003,5\n"},
}


def load_ft(fn):
    b = open(fn, "rb").read()
    nft, nparts = (int(v) for v in np.frombuffer(b, np.uint32, 4)[1:3])
    o = 16
    t, c, v, w = [], [], [], []
    for _ in range(nparts):
        t.append(np.frombuffer(b, np.float64, 1, o)[0]); o += 8
        for _ in range(nft):
            c.append(np.frombuffer(b, np.float64, 3, o)); o += 24
            v.append(np.frombuffer(b, np.float32, 3, o)); o += 12
            w.append(np.frombuffer(b, np.float32, 3, o)); o += 12
    sh = (nparts, nft, 3)
    return np.array(t), np.array(c).reshape(sh), np.array(v).reshape(sh), np.array(w).reshape(sh)


def make(name, dp, step, ddt, boundary, nsteps, keep, extra=(), xml_edit=None):
    out_dir = os.path.join(HERE, "bi4", "flume_" + name)
    os.makedirs(out_dir, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix="flume_")
    try:
        subprocess.check_call([os.path.join(REF, "genflume_ref"), repr(dp), tmp, str(step), str(ddt), "1.0",
                               "CaseFlume", str(boundary)] + list(extra), stdout=subprocess.DEVNULL)
        if xml_edit:
            fx = os.path.join(tmp, "CaseFlume.xml")
            txt = open(fx).read()
            edit = XML_EDITS[xml_edit]
            if isinstance(edit, dict) and "replace" in edit:
                for old, new in edit["replace"]:
                    assert txt.count(old) == 1
                    txt = txt.replace(old, new)
                open(fx, "w").write(txt)
            elif isinstance(edit, dict):  # the <motion> program replaced
                i, j = txt.index("<motion>"), txt.index("</motion>") + len("</motion>")
                open(fx, "w").write(txt[:i] + edit["motion"] + txt[j:])
            else:
                anchor, text = edit if isinstance(edit, tuple) else ("</floating>", edit)
                assert txt.count(anchor) == 1
                open(fx, "w").write(txt.replace(anchor, text + anchor))
        datafiles = DATA_FILES.get(xml_edit, {}) if xml_edit else {}
        for fn, text in datafiles.items():
            open(os.path.join(tmp, fn), "w").write(text)
        files = (["CaseFlume.xml", "CaseFlume.bi4"] + (["CaseFlume_Normals.nbi4"] if boundary == 2 else [])
                 + sorted(datafiles))
        for f in files:
            shutil.copy(os.path.join(tmp, f), os.path.join(out_dir, f))
        out = os.path.join(tmp, "out")
        subprocess.check_call([os.path.join(REF, "DualSPHysics5.2CPU_ref"), os.path.join(tmp, "CaseFlume"), out,
                               "-nsteps:%d" % nsteps, "-svsteps:1", "-nortimes:1", "-saveposdouble:1", "-sv:binx",
                               "-svres:0", "-ompthreads:4"], stdout=subprocess.DEVNULL)
        arrays, times = {}, []
        for part in range(nsteps + 1):
            fn = os.path.join(tmp, "p.bin")
            subprocess.check_call([os.path.join(REF, "partdump_ref"), out, str(part), fn], stdout=subprocess.DEVNULL)
            t, idp, pos, vel, rho = load_dump(fn)
            times.append(t)
            if part in keep:
                arrays.update({"s%d_idp" % part: idp, "s%d_pos" % part: pos, "s%d_vel" % part: vel,
                               "s%d_rhop" % part: rho, "s%d_time" % part: np.float64(t)})
        if os.path.exists(os.path.join(out, "PartFloat.fbi4")):  # (no floating box: nofloat=1)
            subprocess.check_call([os.path.join(REF, "ftdump_ref"), out, os.path.join(tmp, "ft.bin")],
                                  stdout=subprocess.DEVNULL)
            ft, fc, fv, fw = load_ft(os.path.join(tmp, "ft.bin"))
            arrays.update(ft_time=ft, ft_center=fc, ft_fvel=fv, ft_fomega=fw)
        arrays.update(times=np.array(times), meta=np.array([dp, step, ddt, nsteps, boundary], np.float64))
        np.savez_compressed(os.path.join(out_dir, "ref.npz"), **arrays)
        print(name, "ok", sorted(os.listdir(out_dir)))
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    only = sys.argv[1] if len(sys.argv) > 1 else None
    for k, v in VARIANTS.items():
        if only is None or k == only:
            make(k, *v)
