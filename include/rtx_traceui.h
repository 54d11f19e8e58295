/* rtx_traceui.h — the reference-side adapter: RtxRenderParams from the
 * reference's own TraceUI flags (ray/src/ui/TraceUI.h:34-129), for a
 * RayTracer::traceImage (ray/src/RayTracer.cpp:279-314) that forwards to
 * rtx_render instead of running its OpenMP pixel loop.
 *
 * Header-only C++ template over the UI type; the maintainer's RayTracer.cpp
 * includes TraceUI.h first and calls rtx_params_from_traceui(*traceUI, w, h).
 * tests/native/traceui_adapter_check.cpp instantiates it against the
 * UNMODIFIED /root/reference/ray/src/ui/TraceUI.h (the build container only),
 * so the accessor names and types below are the reference's.
 *
 * Mapping (TraceUI accessor -> field):
 *   getDepth()                       -> depth       (-r)
 *   getAAMode()  NONE/SUPERSAMPLE/ADAPTIVE/JITTERED
 *                                    -> aa_mode     (-O a/j/r; RTX_AA_* have the enum's values)
 *   getAASamples()                   -> aa_samples  (-A after a/j/r)
 *   getAAThresh()                    -> aa_thresh   (-B after a)
 *   getATermThresh()                 -> aterm_thresh (-O c -A x; aTermSwitch() is > 0)
 *   dofSwitch() getDofFD() getDofSubDiv() getDofApSz()
 *                                    -> dof dof_fd dof_div dof_apsz (-O d -A -B -C)
 *   anaglyph()                       -> anaglyph    (-O g)
 *   softShadowRes()                  -> ss_res      (-O s -A n)
 *   overlappingObjects()             -> overlapping (-O o)
 * The cube map (-c) is not a render parameter: it is loaded with the scene
 * (rtx_host_cubemap), as TraceUI::smartLoadCubemap does at start-up.
 * Several TraceUI accessors are non-const (dofSwitch, anaglyph, ...), so the
 * UI is taken by non-const reference. */
#ifndef RTX_TRACEUI_H
#define RTX_TRACEUI_H

#include <cstring>

#include "rtx.h"

template <class UI>
inline RtxRenderParams rtx_params_from_traceui(UI& ui, int width, int height) {
  RtxRenderParams p;
  std::memset(&p, 0, sizeof(p));
  p.width = width;
  p.height = height;
  p.depth = ui.getDepth();
  switch (ui.getAAMode()) {
    case UI::AAMode::SUPERSAMPLE: p.aa_mode = RTX_AA_SUPERSAMPLE; break;
    case UI::AAMode::ADAPTIVE: p.aa_mode = RTX_AA_ADAPTIVE; break;
    case UI::AAMode::JITTERED: p.aa_mode = RTX_AA_JITTERED; break;
    default: p.aa_mode = RTX_AA_NONE; break;
  }
  p.aa_samples = ui.getAASamples();
  p.aa_thresh = ui.getAAThresh();
  p.aterm_thresh = ui.aTermSwitch() ? ui.getATermThresh() : 0.0;
  p.dof = ui.dofSwitch() ? 1 : 0;
  p.dof_fd = ui.getDofFD();
  p.dof_div = ui.getDofSubDiv();
  p.dof_apsz = ui.getDofApSz();
  p.anaglyph = ui.anaglyph() ? 1 : 0;
  p.ss_res = ui.softShadowRes();
  p.overlapping = ui.overlappingObjects() ? 1 : 0;
  p.tile = 0;  /* the whole frame; a rank of a multi-GPU job sets tile/shard/nshards/packed */
  p.shard = 0;
  p.nshards = 1;
  p.packed = 0;
  return p;
}

#endif
