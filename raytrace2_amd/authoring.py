"""Scene authoring: seeded generators for the scene JSON the loader reads.

The reference authors its benchmark scenes with `make_scene.py` (its `Scene` builder,
make_scene.py:12-165, and the generators at :176-336) and draws the random parts from Python's
unseeded global `random`. Here the same scenes come from a builder (`SceneDoc`) and generators that
take an explicit `random.Random`, so a scene is reproducible from its seed:

* `cornell_original()`  == make_scene.py:301-306 (`run_cornell_box_original_scene`), whose output
  the reference ships as data/cornell_original_10000_samples.json;
* `cornell_volume()`    == make_scene.py:309-314, shipped as data/cornell_volume_10000_samples.json;
* `book2_final(rng)`    == make_scene.py:176-229 + :317-321 (400 ground boxes of random height,
  media, a Perlin sphere, 1000 random spheres under one transform); the shipped
  data/book2_final_scene_10000_samples.json is one draw of it;
* `sphere_field(n, rng)`: a stress scene (n random spheres of the four reference materials over a
  ground sphere) for BVH-bound measurements at sizes the reference never authored.

The JSON follows the v2 schema of `SceneLoader::LoadScene` (Serialize.cpp:199-360): `textures`,
`materials`, `primitives` (sphere / quad / box, optional `displacement`, optional
`constant_medium`), `scene` (nodes with `primitive`, `transform`, `children`), `camera`,
`background_color`.

    python -m raytrace2_amd.authoring book2 --seed 7 -o /tmp/book2.json
"""
from __future__ import annotations

import argparse
import json
import random
from typing import Dict, List, Optional, Sequence

Vec = Sequence[float]


def _v(x: Vec) -> List[float]:
    return [v for v in x]


def transform(translation: Optional[Vec] = None, rotation: Optional[Vec] = None,
              scale: Optional[Vec] = None) -> Dict:
    """A node transform (ParseTransform, Serialize.cpp:106-132): rotation = [degrees, axis x, y, z]."""
    t: Dict = {}
    if translation is not None:
        t["translation"] = _v(translation)
    if scale is not None:
        t["scale"] = _v(scale)
    if rotation is not None:
        t["rotation"] = _v(rotation)
    return t


def medium(density: float, albedo: Vec) -> Dict:
    """`constant_medium` of a primitive (Serialize.cpp:321-340: the primitive becomes its boundary)."""
    return {"density": density, "albedo": _v(albedo)}


class SceneDoc:
    """Tables of one scene document; every add returns the index later entries refer to."""

    def __init__(self, *, fov: float = 40, center: Vec = (0, 0, 1), look_at: Vec = (0, 0, 0),
                 width: int = 600, aspect_ratio: float = 1.0, background: Vec = (0, 0, 0)):
        self.textures: List[Dict] = []
        self.materials: List[Dict] = []
        self.primitives: List[Dict] = []
        self.nodes: List[Dict] = []
        self.camera = {"fov": fov, "center": _v(center), "look_at": _v(look_at), "width": width,
                       "aspect_ratio": aspect_ratio}
        self.background = _v(background)

    @staticmethod
    def _push(table: List[Dict], entry: Dict) -> int:
        table.append(entry)
        return len(table) - 1

    # -- materials (Material.hpp:12-65) ------------------------------------------------------
    def lambertian(self, albedo: Vec) -> int:
        return self._push(self.materials, {"type": "lambertian", "albedo": _v(albedo)})

    def metal(self, albedo: Vec, fuzz: float) -> int:
        return self._push(self.materials, {"type": "metal", "albedo": _v(albedo), "fuzz": fuzz})

    def dielectric(self, refraction_index: float) -> int:
        return self._push(self.materials, {"type": "dielectric", "refraction_index": refraction_index})

    def light(self, emit: Vec) -> int:
        return self._push(self.materials, {"type": "diffuse_light", "albedo": _v(emit)})

    def textured(self, tex: int) -> int:
        return self._push(self.materials, {"type": "texture", "tex_idx": tex})

    # -- textures (Texture.hpp:14-39) --------------------------------------------------------
    def noise(self, scale: float, noise_type: int = 1, albedo: Vec = (1, 1, 1)) -> int:
        return self._push(self.textures, {"type": "noise", "scale": scale, "noise_type": noise_type,
                                          "albedo": _v(albedo)})

    # -- primitives --------------------------------------------------------------------------
    def _prim(self, entry: Dict, displacement: Optional[Vec], constant_medium: Optional[Dict]) -> int:
        if displacement is not None:
            entry["displacement"] = _v(displacement)
        if constant_medium is not None:
            entry["constant_medium"] = dict(constant_medium)
        return self._push(self.primitives, entry)

    def sphere(self, center: Vec, radius: float, material: int, *, displacement: Optional[Vec] = None,
               constant_medium: Optional[Dict] = None) -> int:
        return self._prim({"type": "sphere", "center": _v(center), "radius": radius, "material": material},
                          displacement, constant_medium)

    def quad(self, q: Vec, u: Vec, v: Vec, material: int, *, constant_medium: Optional[Dict] = None) -> int:
        return self._prim({"type": "quad", "q": _v(q), "u": _v(u), "v": _v(v), "material": material}, None,
                          constant_medium)

    def box(self, a: Vec, b: Vec, material: int, *, constant_medium: Optional[Dict] = None) -> int:
        return self._prim({"type": "box", "a": _v(a), "b": _v(b), "material": material}, None, constant_medium)

    # -- scene graph (Serialize.cpp:165-197) ---------------------------------------------------
    def node(self, primitive: Optional[int] = None, *, xform: Optional[Dict] = None,
             children: Optional[List[Dict]] = None) -> Dict:
        n: Dict = {}
        if xform is not None:
            n["transform"] = xform
        if primitive is not None:
            n["primitive"] = primitive
        if children is not None:
            n["children"] = children
        self.nodes.append(n)
        return n

    def as_dict(self) -> Dict:
        return {"textures": self.textures, "materials": self.materials, "primitives": self.primitives,
                "scene": self.nodes, "camera": self.camera, "background_color": self.background}

    def dump(self, path: str) -> None:
        with open(path, "w") as f:
            json.dump(self.as_dict(), f, indent=2)


# ---- the reference's scenes ----------------------------------------------------------------
def _cornell_room(doc: SceneDoc) -> None:
    """Five walls and the ceiling light (make_scene.py:258-272)."""
    red = doc.lambertian([0.65, 0.05, 0.05])
    white = doc.lambertian([0.73, 0.73, 0.73])
    green = doc.lambertian([0.12, 0.45, 0.15])
    lamp = doc.light([7, 7, 7])
    for q, u, v, m in (([555, 0, 0], [0, 555, 0], [0, 0, 555], green),
                       ([0, 0, 0], [0, 555, 0], [0, 0, 555], red),
                       ([113, 554, 127], [330, 0, 0], [0, 0, 305], lamp),
                       ([0, 0, 0], [555, 0, 0], [0, 0, 555], white),
                       ([0, 555, 0], [555, 0, 0], [0, 0, 555], white),
                       ([0, 0, 555], [555, 0, 0], [0, 555, 0], white)):
        doc.node(doc.quad(q, u, v, m))


# the two rotated blocks: (translation, rotation, far corner)
_BLOCKS = (([130, 0, 65], [-18, 0, 1, 0], [165, 165, 165]), ([265, 0, 295], [15, 0, 1, 0], [165, 330, 165]))


def _cornell_camera(doc: SceneDoc) -> None:
    doc.camera.update(center=[278, 278, -800], look_at=[278, 278, 0], fov=40)


def cornell_original() -> SceneDoc:
    """Cornell box with two white blocks (make_scene.py:275-286, 301-306)."""
    doc = SceneDoc()
    _cornell_room(doc)
    white = doc.lambertian([0.73, 0.73, 0.73])
    for t, r, b in _BLOCKS:
        doc.node(doc.box([0, 0, 0], b, white), xform=transform(t, r))
    _cornell_camera(doc)
    return doc


def cornell_volume() -> SceneDoc:
    """Cornell box whose blocks are smoke (white, then black), make_scene.py:289-298, 309-314."""
    doc = SceneDoc()
    for (t, r, b), albedo in zip(_BLOCKS, ([1, 1, 1], [0, 0, 0])):
        doc.node(doc.box([0, 0, 0], b, 0, constant_medium=medium(0.01, albedo)), xform=transform(t, r))
    _cornell_room(doc)
    _cornell_camera(doc)
    return doc


def book2_final(rng: random.Random) -> SceneDoc:
    """RTNW final scene (make_scene.py:160-229, 317-321): 20x20 ground boxes of random height, a
    ceiling light, moving / glass / metal spheres, a glass sphere filled with blue smoke, global
    fog, a marble sphere and 1000 random white spheres in a rotated cube."""
    doc = SceneDoc(center=[478, 278, -600], look_at=[278, 278, 0])
    ground = doc.lambertian([0.48, 0.83, 0.53])
    side, w = 20, 100.0
    for i in range(side):
        for j in range(side):
            x0, z0 = -1000.0 + i * w, -1000.0 + j * w
            doc.box([x0, 0.0, z0], [x0 + w, rng.uniform(1, 101), z0 + w], ground)
    doc.quad([123, 554, 147], [300, 0, 0], [0, 0, 265], doc.light([7, 7, 7]))
    doc.sphere([400, 400, 200], 50, doc.lambertian([0.7, 0.3, 0.1]), displacement=[30, 0, 0])
    glass = doc.dielectric(1.5)
    doc.sphere([260, 150, 45], 50, glass)
    doc.sphere([0, 150, 145], 50, doc.metal([0.8, 0.8, 0.9], 1.0))
    doc.sphere([360, 150, 145], 70, glass)
    doc.sphere([360, 150, 145], 70, glass, constant_medium=medium(0.2, [0.2, 0.4, 0.9]))
    doc.sphere([0, 0, 0], 5000, glass, constant_medium=medium(0.0001, [1, 1, 1]))
    doc.sphere([220, 280, 300], 80, doc.textured(doc.noise(0.2, 1)))
    for p in range(len(doc.primitives)):
        doc.node(p)
    white = doc.lambertian([0.73, 0.73, 0.73])
    cube = [doc.sphere([rng.uniform(0, 165) for _ in range(3)], 10, white) for _ in range(1000)]
    doc.node(xform=transform([-100, 270, 395], [15, 0, 1, 0]), children=[{"primitive": p} for p in cube])
    return doc


def sphere_field(n: int, rng: random.Random, extent: float = 100.0) -> SceneDoc:
    """Stress scene: n spheres of radius 0.2-1 scattered over a (2*extent)^2 floor, materials mixed
    like RTIOW book 1 (80% diffuse, 15% metal, 5% glass), one large light above, white sky."""
    doc = SceneDoc(fov=30, center=[0, 0.35 * extent, -1.3 * extent], look_at=[0, 0, 0], aspect_ratio=16 / 9,
                   background=[0.7, 0.8, 1.0])
    doc.node(doc.sphere([0, -100000, 0], 100000, doc.lambertian([0.5, 0.5, 0.5])))
    doc.node(doc.quad([-extent / 4, 4 * extent, -extent / 4], [extent / 2, 0, 0], [0, 0, extent / 2],
                      doc.light([4, 4, 4])))
    glass = doc.dielectric(1.5)
    for _ in range(n):
        r = rng.uniform(0.2, 1.0)
        c = [rng.uniform(-extent, extent), r, rng.uniform(-extent, extent)]
        pick = rng.random()
        if pick < 0.8:
            m = doc.lambertian([rng.random() * rng.random() for _ in range(3)])
        elif pick < 0.95:
            m = doc.metal([rng.uniform(0.5, 1) for _ in range(3)], rng.uniform(0, 0.5))
        else:
            m = glass
        doc.node(doc.sphere(c, r, m))
    return doc


GENERATORS = {
    "cornell_original": lambda rng, n: cornell_original(),
    "cornell_volume": lambda rng, n: cornell_volume(),
    "book2": lambda rng, n: book2_final(rng),
    "sphere_field": lambda rng, n: sphere_field(n, rng),
}


def main(argv: Optional[List[str]] = None) -> None:
    ap = argparse.ArgumentParser(description="write a generated scene JSON")
    ap.add_argument("scene", choices=sorted(GENERATORS))
    ap.add_argument("-o", "--out", required=True)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("-n", type=int, default=10000, help="sphere_field: number of spheres")
    a = ap.parse_args(argv)
    GENERATORS[a.scene](random.Random(a.seed), a.n).dump(a.out)


if __name__ == "__main__":
    main()
