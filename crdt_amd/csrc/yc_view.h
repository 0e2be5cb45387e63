// yc_view.h — host-visible records of the materialised view (written by yc_view.hip, read by the
// host in yc_host.cpp). Plain structs: no HIP types, copied device -> host as is.
#pragma once
#include <cstdint>

namespace yc {

// VS_SET: the record holds a struct (client ids use all 32 bits, so no client value can mark
// an empty record)
enum : uint32_t { VS_DELETED = 1u, VS_COUNTABLE = 2u, VS_ITEM = 4u, VS_SET = 8u };
constexpr uint32_t VK_PSUB = 1u;    // ViewKey::flags: a YMap entry
constexpr uint32_t VNONE = 0xFFFFFFFFu;
struct ViewSeg {             // one item run of a list (or a YMap entry's value: its last element)
  uint32_t client, clock, len;
  uint32_t flags;            // VS_*
  uint32_t ref;              // content ref
  uint32_t b0, b1;           // content element bytes in the batch buffer (0, 0 when deleted)
  uint32_t unit;             // merged-store unit of the first element (nested types link by it)
};
struct ViewKey {             // one live list: a YMap entry (KF_PSUB) or a YArray list
  uint32_t slot, flags;
  uint32_t parent_unit;      // parent type item unit, NONE = root type
  uint32_t name_pos, name_len;   // root type name (root lists)
  uint32_t psub_pos, psub_len;   // YMap entry key
  uint32_t seg0, nseg;       // YArray: members in document order, ViewSeg [seg0, seg0 + nseg)
  ViewSeg win;               // YMap entry: the winning item's value (flags without VS_SET = none)
};

}  // namespace yc
