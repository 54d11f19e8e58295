"""Parity cases: (name, scene, reference CLI flags).  Sizes are small so the
CPU restatement finishes in seconds; each case exercises a reference feature."""

CASES = [
    ("spheres_r5", "spheres_overlap.ray", "-w 64 -r 5"),
    ("distance_r3", "distance.ray", "-w 64 -r 3"),
    ("concrete2_bump", "concrete_2.ray", "-w 64 -r 5"),
    ("concrete1_r1", "concrete_1.ray", "-w 48 -r 1"),
    ("spotlight", "box_cyl_opaque_shadow_spotlight.ray", "-w 64 -r 2"),
    ("lava_arealight", "lava_box.ray", "-w 48 -r 3 -O s -A 4"),
    ("hitchcock_c2", "hitchcock.ray", "-w 64 -r 3 -O r -A 2"),
    ("hitchcock_c1", "hitchcock.ray", "-w 64 -r 1"),
    ("trimesh2_aa", "trimesh2_square.ray", "-w 40 -r 5 -O r -A 2"),
    ("trimesh2_dof", "trimesh2.ray", "-w 48 -r 3 -O d -A 2.5 -B 4 -C 0.05"),
    ("hitchcock_adaptive", "hitchcock.ray", "-w 24 -r 2 -O a -A 3 -B 0.02"),
    ("spheres_anaglyph", "spheres_overlap.ray", "-w 48 -r 3 -O g"),
    ("spheres_aterm", "spheres_overlap.ray", "-w 48 -r 5 -O c -A 0.01"),
    ("spheres_r0", "spheres_overlap.ray", "-w 32 -r 0"),
    ("distance_aa3", "distance.ray", "-w 24 -r 2 -O r -A 3"),
    ("cones_r4", "cones.ray", "-w 64 -r 4"),
    ("cones_aa", "cones.ray", "-w 32 -r 3 -O r -A 2"),
    # -c: relative cube-map paths name files under tests/golden
    ("cubemap_cones", "cones.ray", "-w 48 -r 3 -c cubemap/posx.bmp"),
    ("cubemap_spheres_aa", "spheres_overlap.ray", "-w 32 -r 4 -O r -A 2 -c cubemap/negz.bmp"),
    ("cubemap_r0", "cones.ray", "-w 24 -r 0 -c cubemap/posy.bmp"),
    # -O o: discoverMat media on refraction and along shadow walks
    ("overlap_spheres", "spheres_overlap.ray", "-w 48 -r 5 -O o"),
    ("overlap_cones", "cones.ray", "-w 40 -r 4 -O o"),
    ("overlap_hitchcock", "hitchcock.ray", "-w 40 -r 3 -O o"),
    ("overlap_trimesh_aa", "trimesh2_square.ray", "-w 24 -r 3 -O o -O r -A 2"),
    ("overlap_area_cube", "lava_box.ray", "-w 32 -r 3 -O o -O s -A 4 -c cubemap/posz.bmp"),
    # BASELINE.json configs at parity size: C3 (1024^2 square trimesh2,
    # 4x4 regular AA, depth 5), the headline (16:9 trimesh2, 4x4 AA, depth
    # 5) and C4 (DoF x16, focal 2.5, aperture 0.05, depth 5)
    ("c3_trimesh2_aa4", "trimesh2_square.ray", "-w 32 -r 5 -O r -A 4"),
    ("headline_aa4", "trimesh2.ray", "-w 32 -r 5 -O r -A 4"),
    ("c4_dof16", "trimesh2.ray", "-w 32 -r 5 -O d -A 2.5 -B 16 -C 0.05"),
    # next-tier rows: area_light_circ, per-vertex materials, composed
    # transforms, quaternion camera, PNG textures + bump
    ("circ_light", "circ_light.ray", "-w 40 -r 3 -O s -A 5"),
    ("vmats", "vmats.ray", "-w 40 -r 4"),
    ("xforms_aa", "xforms.ray", "-w 48 -r 4 -O r -A 2"),
    ("xforms_quat", "xforms_quat.ray", "-w 32 -r 3"),
    ("png_tex", "png_tex.ray", "-w 40 -r 2"),
    # the composed-transform and per-vertex-material known-answer scenes
    ("kat_xform_nested", "xform_nested.ray", "-w 24 -r 1"),
    ("kat_xform_matrix", "xform_matrix.ray", "-w 24 -r 1"),
    ("kat_vmat_quad", "vmat_quad.ray", "-w 16 -r 0"),
    # recursion deeper than the old -r 16 cap (RayTracer.cpp:108-174 is
    # unbounded): 2.3 M secondary rays in a 16 x 16 frame
    ("spheres_deep_r20", "spheres_overlap.ray", "-w 16 -r 20"),
    ("circ_deep_r40", "circ_light.ray", "-w 16 -r 40"),
    # adaptive AA on the wavefront path (adapt_*_kernel): subdivision levels
    # on a trimesh frame with fused walks and ray-tree buckets, with the DoF
    # camera-ray split, and with -O g (adaptaa calls trace(): no anaglyph eye)
    ("trimesh2_adaptive", "trimesh2.ray", "-w 32 -r 5 -O a -A 4 -B 0.03"),
    ("adaptive_dof", "trimesh2.ray", "-w 24 -r 3 -O a -A 2 -B 0.05 -O d -A 2.5 -B 4 -C 0.05"),
    ("adaptive_anaglyph", "spheres_overlap.ray", "-w 24 -r 3 -O g -O a -A 2 -B 0.05"),
    # shadow walks ending at objects opaque to them (walk_hit's shortcut):
    # exits from inside an opaque box, a coincident second box (exits at the
    # same t), an opaque cube inside a glass sphere
    ("walk_opaque", "walk_opaque.ray", "-w 32 -r 4"),
    ("walk_opaque_aa", "walk_opaque.ray", "-w 24 -r 5 -O r -A 2"),
    # R1 at parity size: the headline geometry with reflective / transmissive
    # materials (ray trees that fork at every level, RayTracer.cpp:127-165)
    ("r1_glass_aa4", "trimesh2_glass.ray", "-w 32 -r 5 -O r -A 4"),
    ("r1_glass_r8", "trimesh2_glass.ray", "-w 40 -r 8"),
]
