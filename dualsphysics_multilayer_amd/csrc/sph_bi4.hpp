// sph_bi4.hpp — the DualSPHysics binary container (.bi4) and its PART / case layout
// (SURVEY.md §8(f) row 2).  Host-only C++.
//
// Container (restated from the reference's reader/writer, JBinaryData.cpp:700-1160,
// 1467-1545; JBinaryData.h:68-76,160-176):
//   header, 64 B: title[60] = "#FileJBD " + file code, space-padded to 58 chars, '\n',
//                 0; byte order (0 little endian); 3 unused bytes
//   item        := u32 def_size, def, [values], arrays..., items...
//   def         := str "\nITEM\n", str name, bool hide, bool hide_values, str fmt_float,
//                  str fmt_double, u32 n_arrays, u32 n_items, u32 values_size
//   values      := str "\nVALUES", u32 n, { str name, i32 type, payload }   (values_size B)
//   array       := u32 def_size, str "\nARRAY", str name, bool hide, i32 type, u32 count,
//                  u32 data_size, data (text arrays: str per element)
//   str := u32 length + bytes;  bool := i32 (0/1)
//   types (JBinaryDataDef::TpData): 1 text, 2 bool, 3 char, 4 uchar, 5 short, 6 ushort,
//   7 int, 8 uint, 9 llong, 10 ullong, 11 float, 12 double, 20 int3, 21 uint3,
//   22 float3, 23 double3.
// PART / case file (JPartDataBi4.cpp:183-440): file code "JPartDataBi4"; the root item
// carries the case values (Piece, Npiece, RunCode, ..., CaseNp, Dp, H, B, ..., MapPosMin,
// PeriMode, ...), one child item "PART_%04u" carries the part values (Cpart, TimeStep,
// Npok, Nout, Step, RunTime, DomainMin/Max, [SymplecticDtPre]) and the particle arrays
// Idp (uint), Posd (double3) or Pos (float3), Vel (float3), Rhop (float).
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace sphx {
namespace bi4 {

enum Type : int32_t {
  Text = 1, Bool = 2, Char = 3, Uchar = 4, Short = 5, Ushort = 6, Int = 7, Uint = 8, Llong = 9, Ullong = 10,
  Float = 11, Double = 12, Int3 = 20, Uint3 = 21, Float3 = 22, Double3 = 23
};
size_t type_size(int32_t t);  // bytes per element, 0 for text / unknown

struct Value {
  std::string name;
  int32_t type = 0;
  std::vector<uint8_t> bytes;  // raw payload (text: the characters)
};
struct Array {
  std::string name;
  bool hide = false;
  int32_t type = 0;
  uint32_t count = 0;
  std::vector<uint8_t> bytes;  // count * type_size (text arrays are not used here)
};
struct Item {
  std::string name;
  bool hide = false, hide_values = false;
  std::string fmt_float = "%.7E", fmt_double = "%.15E";
  std::vector<Value> values;
  std::vector<Array> arrays;
  std::vector<Item> items;

  const Value* value(const std::string& n) const;
  const Array* array(const std::string& n) const;
  const Item* item_prefix(const std::string& prefix) const;
  void set(const std::string& n, int32_t type, const void* data, size_t bytes);
  void set_text(const std::string& n, const std::string& v) { set(n, Text, v.data(), v.size()); }
  template <class T>
  void set_pod(const std::string& n, int32_t type, const T& v) { set(n, type, &v, sizeof(T)); }
  void add_array(const std::string& n, int32_t type, uint32_t count, const void* data);
  double get_double(const std::string& n, double def) const;
  uint64_t get_uint(const std::string& n, uint64_t def) const;
  bool get_bool(const std::string& n, bool def) const;
  std::string get_text(const std::string& n, const std::string& def) const;
  bool get_double3(const std::string& n, double out[3]) const;
};

// Read / write a whole container file; `filecode` is checked against the header title.
Item read_file(const std::string& path, const std::string& filecode);
void write_file(const std::string& path, const std::string& filecode, const Item& root);
// A list file (JBinaryData::SaveFileListApp / LoadFileListApp): head item then items appended
// after it; read back as [head, item 1, ...].
std::vector<Item> read_list_file(const std::string& path, const std::string& filecode);
void write_list_file(const std::string& path, const std::string& filecode, const Item& head,
                     const std::vector<Item>& items);

}  // namespace bi4
}  // namespace sphx
