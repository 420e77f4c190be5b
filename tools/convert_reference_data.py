#!/usr/bin/env python
"""Convert the reference's gait10dof18musc model and data files into the
committed data files under opensim-moco_amd/mocohip/data/ (run once, in the
container that has /root/reference; the GPU box never reads the reference).

Inputs (all under /root/reference, read as data):
  Moco/Archive/Tests/testGait10dof18musc_subject01.osim   (model)
  Moco/Tests/walk_gait1018_subject01_grf.mot               (GRF data)
  Moco/Tests/walk_gait1018_subject01_grf.xml               (ExternalLoads)
  Moco/Tests/walk_gait1018_state_reference.mot             (MocoTrack reference)
  Moco/Tests/std_testMocoTrackGait10dof18musc_solution.sto (golden solution)
  Moco/Tests/std_testMocoInverse_subject_18musc_solution.sto (MocoInverse
      golden solution: its initial row pins the initial-activation endpoint
      constraint, MocoInverse.cpp:93; the whole solution pins the Rajagopal
      18-muscle model's wrapping, couplers and dynamics at solution level)
  Moco/Tests/subject_walk_armless_18musc.osim, subject_walk_armless_coordinates.mot,
      subject_walk_armless_grfs.mot, subject_walk_armless_external_loads.xml
      (testMocoInverse.cpp:118-147)
  Moco/Examples/C++/example3DWalking/subject_walk_armless.osim (80 muscles,
      BASELINE configs[3])
"""
import json
import math
import os
import sys
import xml.etree.ElementTree as ET

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "opensim-moco_amd"))

from mocohip.model import model_to_dict  # noqa: E402
from mocohip.osim import read_osim, read_storage  # noqa: E402

REF = "/root/reference"
DATA = os.path.join(REPO, "opensim-moco_amd", "mocohip", "data")
GOLDEN = os.path.join(REPO, "tests", "golden")


def main():
    os.makedirs(DATA, exist_ok=True)
    os.makedirs(GOLDEN, exist_ok=True)
    osim = os.path.join(REF, "Moco/Archive/Tests/testGait10dof18musc_subject01.osim")
    model = read_osim(osim)
    with open(os.path.join(DATA, "gait10dof18musc.json"), "w") as fh:
        json.dump(model_to_dict(model), fh, indent=1)

    # Ground reactions (ExternalLoads file: which columns go to which body).
    labels, data, hdr = read_storage(os.path.join(REF, "Moco/Tests/walk_gait1018_subject01_grf.mot"))
    xml = ET.parse(os.path.join(REF, "Moco/Tests/walk_gait1018_subject01_grf.xml")).getroot()
    forces = []
    for ef in xml.iter("ExternalForce"):
        forces.append({
            "name": ef.get("name"),
            "body": ef.findtext("applied_to_body").strip(),
            "force_expressed_in_body": ef.findtext("force_expressed_in_body").strip(),
            "point_expressed_in_body": ef.findtext("point_expressed_in_body").strip(),
            "force_identifier": ef.findtext("force_identifier").strip(),
            "point_identifier": ef.findtext("point_identifier").strip(),
            "torque_identifier": ef.findtext("torque_identifier").strip(),
        })
    grf = {"labels": labels, "time": data[:, 0].tolist(),
           "columns": {l: data[:, i].tolist() for i, l in enumerate(labels) if i > 0},
           "external_forces": forces}
    with open(os.path.join(DATA, "walk_gait1018_subject01_grf.json"), "w") as fh:
        json.dump(grf, fh)

    # State reference (degrees -> radians for rotational coordinates, as
    # TableProcessor does for inDegrees=yes tables).
    labels, data, hdr = read_storage(os.path.join(REF, "Moco/Tests/walk_gait1018_state_reference.mot"))
    rot = {c.path + "/value" for j in model.joints for c in j.coordinates
           if c.motion_type == "rotational"}
    in_deg = hdr.get("inDegrees", "no").lower() == "yes"
    cols = {}
    for i, l in enumerate(labels):
        if i == 0:
            continue
        v = data[:, i]
        if in_deg and l in rot:
            v = v * math.pi / 180.0
        cols[l] = v.tolist()
    with open(os.path.join(DATA, "walk_gait1018_state_reference.json"), "w") as fh:
        json.dump({"time": data[:, 0].tolist(), "columns": cols}, fh)

    # Golden torque-driven MocoTrack solution (N=65 HS; 131 rows).
    labels, data, hdr = read_storage(os.path.join(REF, "Moco/Tests/std_testMocoTrackGait10dof18musc_solution.sto"))
    np.savez_compressed(os.path.join(GOLDEN, "std_testMocoTrackGait10dof18musc_solution.npz"),
                        labels=np.array(labels), data=data,
                        header=np.array([f"{k}={v}" for k, v in hdr.items()]))
    # MocoInverse golden solution (Rajagopal 18 muscles, N=11): the initial
    # row's excitation / activation pairs of every muscle
    labels, data, hdr = read_storage(os.path.join(REF, "Moco/Tests/std_testMocoInverse_subject_18musc_solution.sto"))
    col = {l: i for i, l in enumerate(labels)}
    mus = [l[:-len("/activation")] for l in labels if l.endswith("/activation")
           and l[:-len("/activation")] in col]
    np.savez_compressed(os.path.join(GOLDEN, "inverse_initial_activation.npz"),
                        muscles=np.array(mus),
                        excitation=np.array([data[0, col[m]] for m in mus]),
                        activation=np.array([data[0, col[m + "/activation"]] for m in mus]),
                        time=data[0, 0],
                        header=np.array([f"{k}={v}" for k, v in hdr.items()]))
    # Rajagopal 2016 models (SURVEY §8 X1 / configs[3], and the MocoInverse
    # 18-muscle test model with its golden solution), kinematics, GRFs
    raja = [("rajagopal18.json", "Moco/Tests/subject_walk_armless_18musc.osim"),
            ("rajagopal80.json", "Moco/Examples/C++/example3DWalking/subject_walk_armless.osim")]
    for out, src in raja:
        # the models as written (PathWrapSets kept on the muscles); the
        # configs drop them where replaceMuscles does (configs._replaced)
        with open(os.path.join(DATA, out), "w") as fh:
            json.dump(model_to_dict(read_osim(os.path.join(REF, src), keep_path_wraps=True)), fh)
    labels, data, hdr = read_storage(os.path.join(REF, "Moco/Tests/subject_walk_armless_coordinates.mot"))
    r18 = read_osim(os.path.join(REF, "Moco/Tests/subject_walk_armless_18musc.osim"))
    rot = {c.name for j in r18.joints for c in j.coordinates if c.motion_type == "rotational"}
    in_deg = hdr.get("inDegrees", "no").lower() == "yes"
    cols = {}
    for i, l in enumerate(labels):
        if i == 0:
            continue
        v = data[:, i]
        if in_deg and l in rot:     # TableProcessor::processAndConvertToRadians
            v = v * math.pi / 180.0
        cols[l] = v.tolist()
    with open(os.path.join(DATA, "subject_walk_armless_coordinates.json"), "w") as fh:
        json.dump({"time": data[:, 0].tolist(), "columns": cols}, fh)
    labels, data, hdr = read_storage(os.path.join(REF, "Moco/Tests/subject_walk_armless_grfs.mot"))
    xml = ET.parse(os.path.join(REF, "Moco/Tests/subject_walk_armless_external_loads.xml")).getroot()
    forces = []
    for ef in xml.iter("ExternalForce"):
        forces.append({k: ef.findtext(k).strip() for k in (
            "applied_to_body", "force_expressed_in_body", "point_expressed_in_body",
            "force_identifier", "point_identifier", "torque_identifier")})
        forces[-1]["name"] = ef.get("name")
        forces[-1]["body"] = forces[-1].pop("applied_to_body")
    with open(os.path.join(DATA, "subject_walk_armless_grf.json"), "w") as fh:
        json.dump({"labels": labels, "time": data[:, 0].tolist(),
                   "columns": {l: data[:, i].tolist() for i, l in enumerate(labels) if i > 0},
                   "external_forces": forces}, fh)
    labels, data, hdr = read_storage(os.path.join(REF, "Moco/Tests/std_testMocoInverse_subject_18musc_solution.sto"))
    np.savez_compressed(os.path.join(GOLDEN, "std_testMocoInverse_subject_18musc_solution.npz"),
                        labels=np.array(labels), data=data,
                        header=np.array([f"{k}={v}" for k, v in hdr.items()]))
    print("wrote", DATA, GOLDEN)


if __name__ == "__main__":
    main()
