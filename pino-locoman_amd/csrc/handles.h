// Host-side handle types shared by the C-ABI translation units (not part of the ABI).
#pragma once
#include <string.h>

#include <vector>

#include "model.h"

struct pl_model {
  PlModel m;
  int nframes;
  std::vector<int> frame_parent;
  std::vector<double> frame_R, frame_p;
};

// Placement of frame `fid` w.r.t. its parent joint (model.frames[fid]); invalid ids
// (e.g. getFrameId of an absent name, which pinocchio returns as nframes) give valid = 0.
inline PlFrameRef frame_ref(const pl_model* M, int fid) {
  PlFrameRef f;
  memset(&f, 0, sizeof(f));
  if (fid < 0 || fid >= M->nframes) { f.valid = 0; f.joint = -1; return f; }
  f.valid = 1;
  f.joint = M->frame_parent[fid];
  for (int k = 0; k < 9; ++k) f.R[k] = M->frame_R[9 * fid + k];
  for (int k = 0; k < 3; ++k) f.p[k] = M->frame_p[3 * fid + k];
  return f;
}

void pl_set_error(const char* fmt, ...);
