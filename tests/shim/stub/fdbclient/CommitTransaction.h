// Minimal stand-ins for the flow / fdbclient types that fdbserver/ConflictSet.h
// names, so the drop-in TU (foundationdb_amd/shim/ConflictSetShim.cpp) can be
// compiled and exercised outside an fdbserver build tree.  Only the members
// the shim uses exist: KeyRangeRef::{begin,end} (fdbclient/FDBTypes.h:161),
// StringRef::{begin(),size()} (flow/Arena.h), CommitTransactionRef::
// {read_conflict_ranges, write_conflict_ranges, read_snapshot}, Arena
// (fdbclient/CommitTransaction.h:89-121).  Test infrastructure only.
#pragma once
#include <cstddef>
#include <cstdint>
#include <utility>
#include <vector>
using namespace std;

typedef int64_t Version;

struct StringRef {
    const uint8_t* data = nullptr;
    int length = 0;
    StringRef() = default;
    StringRef(const uint8_t* d, int l) : data(d), length(l) {}
    const uint8_t* begin() const { return data; }
    int size() const { return length; }
};
typedef StringRef KeyRef;

struct KeyRangeRef {
    KeyRef begin, end;
    KeyRangeRef() = default;
    KeyRangeRef(KeyRef b, KeyRef e) : begin(b), end(e) {}
};

struct Arena {};  // (flow/Arena.h: the owner of a request's memory)

template <class T>
struct VectorRef {
    std::vector<T> items;
    const T* begin() const { return items.data(); }
    const T* end() const { return items.data() + items.size(); }
    int size() const { return (int)items.size(); }
    void push_back(const T& x) { items.push_back(x); }
    void push_back(Arena&, const T& x) { items.push_back(x); }  // (flow/Arena.h VectorRef::push_back)
};

template <class T>
struct Standalone : T {};

struct CommitTransactionRef {
    VectorRef<KeyRangeRef> read_conflict_ranges;
    VectorRef<KeyRangeRef> write_conflict_ranges;
    Version read_snapshot = 0;
};
