// Shared-memory object store (the plasma-store equivalent of the runtime).
//
// One arena per (virtual) node: a file in /dev/shm mapped by every process of the node.
// Layout: [Header | Slot table | data region]. The header holds a process-shared *robust*
// mutex (a process that dies holding it does not wedge the node), a first-fit free list with
// coalescing over the data region, and an open-addressed slot table keyed by the 32-char
// object id. Objects are created (allocated), filled in place by the writer (Arrow IPC is
// serialised straight into the arena: no intermediate copy), sealed, then read zero-copy by
// any process that maps the arena. Readers pin objects with a reference count; deleting a
// pinned object defers the free until the last release.
//
// Reference role: Ray's plasma object store holding Arrow blocks
// (python/raydp/spark/dataset.py:54-84, :222); the JVM side's ObjectRefHolder pinning
// (core/raydp-main/src/main/scala/org/apache/spark/sql/raydp/ObjectStoreWriter.scala:232-271).
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <new>

namespace {

constexpr uint64_t kMagic = 0x5244504F424A5354ULL;  // "RDPOBJST"
constexpr int kIdLen = 32;
constexpr uint64_t kAlign = 64;

enum SlotState : int32_t { kEmpty = 0, kCreated = 1, kSealed = 2, kTomb = 3 };

struct Slot {
  char id[kIdLen];
  uint64_t off;
  uint64_t size;     // requested bytes
  uint64_t alloc;    // allocated bytes (aligned)
  int32_t state;
  int32_t refcnt;
  int32_t kind;
  int32_t pending_delete;
  int64_t owner_pid;
};

struct FreeBlock {
  uint64_t size;
  uint64_t next;  // offset (relative to data start) of next free block, or UINT64_MAX
};

struct Header {
  uint64_t magic;
  uint64_t capacity;   // data region bytes
  uint64_t data_off;   // offset of the data region from the mapping start
  uint32_t nslots;
  uint32_t count;
  uint64_t used;
  uint64_t free_head;  // relative offset of first free block, UINT64_MAX if none
  uint64_t total_size;
  pthread_mutex_t mu;
};

struct Store {
  int fd;
  uint8_t* base;
  uint64_t map_size;
  Header* h;
  Slot* slots;
  uint8_t* data;
};

constexpr uint64_t kNil = UINT64_MAX;

inline uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

uint64_t hash_id(const char* id) {
  uint64_t h = 1469598103934665603ULL;
  for (int i = 0; i < kIdLen && id[i]; ++i) h = (h ^ (uint8_t)id[i]) * 1099511628211ULL;
  return h;
}

class Lock {
 public:
  explicit Lock(Header* h) : h_(h) {
    int rc = pthread_mutex_lock(&h_->mu);
    if (rc == EOWNERDEAD) pthread_mutex_consistent(&h_->mu);
  }
  ~Lock() { pthread_mutex_unlock(&h_->mu); }

 private:
  Header* h_;
};

FreeBlock* fb(Store* s, uint64_t rel) { return reinterpret_cast<FreeBlock*>(s->data + rel); }

// first fit; returns relative offset or kNil
uint64_t alloc_block(Store* s, uint64_t* need_io) {
  uint64_t need = *need_io;
  uint64_t prev = kNil, cur = s->h->free_head;
  while (cur != kNil) {
    FreeBlock* b = fb(s, cur);
    if (b->size >= need) {
      uint64_t rest = b->size - need;
      uint64_t next = b->next;
      if (rest >= kAlign * 2) {
        uint64_t tail = cur + need;
        FreeBlock* t = fb(s, tail);
        t->size = rest;
        t->next = next;
        next = tail;
      } else {
        need = b->size;
      }
      if (prev == kNil) s->h->free_head = next; else fb(s, prev)->next = next;
      s->h->used += need;
      *need_io = need;
      return cur;
    }
    prev = cur;
    cur = b->next;
  }
  return kNil;
}

void free_block(Store* s, uint64_t off, uint64_t size) {
  s->h->used -= size;
  // insert sorted by offset, coalesce with neighbours
  uint64_t prev = kNil, cur = s->h->free_head;
  while (cur != kNil && cur < off) {
    prev = cur;
    cur = fb(s, cur)->next;
  }
  FreeBlock* nb = fb(s, off);
  nb->size = size;
  nb->next = cur;
  if (prev == kNil) s->h->free_head = off; else fb(s, prev)->next = off;
  if (cur != kNil && off + nb->size == cur) {
    nb->size += fb(s, cur)->size;
    nb->next = fb(s, cur)->next;
  }
  if (prev != kNil) {
    FreeBlock* pb = fb(s, prev);
    if (prev + pb->size == off) {
      pb->size += nb->size;
      pb->next = nb->next;
    }
  }
}

Slot* find_slot(Store* s, const char* id, bool for_insert) {
  const uint32_t n = s->h->nslots;
  uint64_t i = hash_id(id) % n;
  Slot* tomb = nullptr;
  for (uint32_t probe = 0; probe < n; ++probe, i = (i + 1) % n) {
    Slot* sl = &s->slots[i];
    if (sl->state == kEmpty) return for_insert ? (tomb ? tomb : sl) : nullptr;
    if (sl->state == kTomb) {
      if (for_insert && !tomb) tomb = sl;
      continue;
    }
    if (strncmp(sl->id, id, kIdLen) == 0) return sl;
  }
  return for_insert ? tomb : nullptr;
}

void release_slot(Store* s, Slot* sl) {
  free_block(s, sl->off, sl->alloc);
  sl->state = kTomb;
  sl->refcnt = 0;
  sl->pending_delete = 0;
  s->h->count--;
}

}  // namespace

extern "C" {

void* rt_store_create(const char* path, uint64_t capacity, uint32_t nslots) {
  capacity = align_up(capacity, kAlign);
  if (nslots < 64) nslots = 64;
  uint64_t hdr = align_up(sizeof(Header) + sizeof(Slot) * (uint64_t)nslots, 4096);
  uint64_t total = hdr + capacity;
  int fd = open(path, O_RDWR | O_CREAT | O_EXCL, 0600);
  if (fd < 0) return nullptr;
  if (ftruncate(fd, (off_t)total) != 0) {
    close(fd);
    unlink(path);
    return nullptr;
  }
  void* m = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (m == MAP_FAILED) {
    close(fd);
    unlink(path);
    return nullptr;
  }
  Store* s = new (std::nothrow) Store{fd, (uint8_t*)m, total, (Header*)m, nullptr, nullptr};
  Header* h = s->h;
  memset(h, 0, sizeof(Header));
  h->capacity = capacity;
  h->data_off = hdr;
  h->nslots = nslots;
  h->total_size = total;
  pthread_mutexattr_t a;
  pthread_mutexattr_init(&a);
  pthread_mutexattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
  pthread_mutexattr_setrobust(&a, PTHREAD_MUTEX_ROBUST);
  pthread_mutex_init(&h->mu, &a);
  pthread_mutexattr_destroy(&a);
  s->slots = reinterpret_cast<Slot*>(s->base + sizeof(Header));
  memset(s->slots, 0, sizeof(Slot) * (uint64_t)nslots);
  s->data = s->base + hdr;
  FreeBlock* b = reinterpret_cast<FreeBlock*>(s->data);
  b->size = capacity;
  b->next = kNil;
  h->free_head = 0;
  std::atomic_thread_fence(std::memory_order_release);
  h->magic = kMagic;
  return s;
}

void* rt_store_open(const char* path) {
  int fd = open(path, O_RDWR);
  if (fd < 0) return nullptr;
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    return nullptr;
  }
  void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (m == MAP_FAILED) {
    close(fd);
    return nullptr;
  }
  Store* s = new (std::nothrow) Store{fd, (uint8_t*)m, (uint64_t)st.st_size, (Header*)m, nullptr, nullptr};
  if (s->h->magic != kMagic) {
    munmap(m, (size_t)st.st_size);
    close(fd);
    delete s;
    return nullptr;
  }
  s->slots = reinterpret_cast<Slot*>(s->base + sizeof(Header));
  s->data = s->base + s->h->data_off;
  return s;
}

void rt_store_close(void* hs) {
  Store* s = (Store*)hs;
  if (!s) return;
  munmap(s->base, s->map_size);
  close(s->fd);
  delete s;
}

int rt_store_unlink(const char* path) { return unlink(path); }

uint8_t* rt_store_data(void* hs) { return ((Store*)hs)->data; }
uint64_t rt_store_capacity(void* hs) { return ((Store*)hs)->h->capacity; }

// Allocate an object; returns the data-relative offset, or
// -1 out of memory, -2 id already present, -3 slot table full.
int64_t rt_obj_create(void* hs, const char* id, uint64_t size, int32_t kind, int64_t pid) {
  Store* s = (Store*)hs;
  Lock l(s->h);
  if (find_slot(s, id, false) != nullptr) return -2;
  Slot* sl = find_slot(s, id, true);
  if (sl == nullptr) return -3;
  uint64_t need = align_up(size ? size : 1, kAlign);
  uint64_t got = need;  // alloc_block may widen it to absorb an unsplittable remnant
  uint64_t off = alloc_block(s, &got);
  if (off == kNil) return -1;
  memset(sl->id, 0, kIdLen);
  strncpy(sl->id, id, kIdLen);
  sl->off = off;
  sl->size = size;
  sl->alloc = got;
  sl->state = kCreated;
  sl->refcnt = 1;  // the creator's pin until seal/release
  sl->kind = kind;
  sl->pending_delete = 0;
  sl->owner_pid = pid;
  s->h->count++;
  return (int64_t)off;
}

int rt_obj_seal(void* hs, const char* id) {
  Store* s = (Store*)hs;
  Lock l(s->h);
  Slot* sl = find_slot(s, id, false);
  if (!sl || sl->state != kCreated) return -1;
  sl->state = kSealed;
  sl->refcnt -= 1;
  return 0;
}

// Pin + locate a sealed object: 0 ok, -1 missing, -3 not yet sealed.
int rt_obj_get(void* hs, const char* id, uint64_t* off, uint64_t* size, int32_t* kind) {
  Store* s = (Store*)hs;
  Lock l(s->h);
  Slot* sl = find_slot(s, id, false);
  if (!sl || sl->pending_delete) return -1;
  if (sl->state != kSealed) return -3;
  sl->refcnt += 1;
  *off = sl->off;
  *size = sl->size;
  *kind = sl->kind;
  return 0;
}

int rt_obj_contains(void* hs, const char* id) {
  Store* s = (Store*)hs;
  Lock l(s->h);
  Slot* sl = find_slot(s, id, false);
  return sl && sl->state == kSealed && !sl->pending_delete ? 1 : 0;
}

int rt_obj_release(void* hs, const char* id) {
  Store* s = (Store*)hs;
  Lock l(s->h);
  Slot* sl = find_slot(s, id, false);
  if (!sl) return -1;
  if (sl->refcnt > 0) sl->refcnt -= 1;
  if (sl->refcnt == 0 && sl->pending_delete) release_slot(s, sl);
  return 0;
}

int rt_obj_delete(void* hs, const char* id) {
  Store* s = (Store*)hs;
  Lock l(s->h);
  Slot* sl = find_slot(s, id, false);
  if (!sl) return -1;
  if (sl->refcnt > 0) {
    sl->pending_delete = 1;
    return 1;
  }
  release_slot(s, sl);
  return 0;
}

// Abort an unsealed creation (writer failed).
int rt_obj_abort(void* hs, const char* id) {
  Store* s = (Store*)hs;
  Lock l(s->h);
  Slot* sl = find_slot(s, id, false);
  if (!sl || sl->state != kCreated) return -1;
  release_slot(s, sl);
  return 0;
}

void rt_store_stats(void* hs, uint64_t* used, uint64_t* capacity, uint64_t* count) {
  Store* s = (Store*)hs;
  Lock l(s->h);
  *used = s->h->used;
  *capacity = s->h->capacity;
  *count = s->h->count;
}

// Copy up to `max` sealed ids (32 chars each, not NUL-terminated) into out; returns count.
int rt_store_list(void* hs, char* out, int max) {
  Store* s = (Store*)hs;
  Lock l(s->h);
  int n = 0;
  for (uint32_t i = 0; i < s->h->nslots && n < max; ++i) {
    Slot* sl = &s->slots[i];
    if (sl->state == kSealed && !sl->pending_delete) {
      memcpy(out + (size_t)n * kIdLen, sl->id, kIdLen);
      ++n;
    }
  }
  return n;
}

}  // extern "C"
