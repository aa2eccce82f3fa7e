/*
 * pip_shm.h -- layout of the shared-memory world segment that bin/mpiexec
 * creates and every rank (pip_world.c) attaches: a header, one 64-byte
 * mailbox slot per rank, then one PIP_CHUNK data area per rank.
 */
#ifndef PIP_SHM_H_INCLUDED
#define PIP_SHM_H_INCLUDED

#include <stdatomic.h>
#include <stdint.h>

#define PIP_MAGIC       0x50495057u      /* "PIPW" */
#define PIP_MAX_RANKS   64
#define PIP_CHUNK       ((size_t) 1 << 20)

/* `owner` is the whole hand-over state in ONE word: 0 = the data area is free,
 * dst + 1 = it holds a chunk for rank dst.  A receiver matches its own rank and
 * acquires the chunk with a single load; a separate (full, dst) pair could be
 * read across a recycle of the slot for another destination and lose a chunk. */
typedef struct {
    _Atomic uint32_t owner;
    uint32_t bytes;             /* this chunk's bytes */
    uint64_t total;             /* the whole message's bytes (every chunk carries it) */
    char pad[48];
} pip_slot_t;

typedef struct {
    uint32_t magic;
    uint32_t size;              /* number of ranks */
    char pad[56];
    pip_slot_t slot[PIP_MAX_RANKS];
} pip_shm_t;

/* data areas start page-aligned after the header */
#define PIP_DATA_OFFSET (((sizeof(pip_shm_t)) + 4095) & ~(size_t) 4095)
#define PIP_SEGMENT_BYTES(n) (PIP_DATA_OFFSET + (size_t) (n) * PIP_CHUNK)

#endif /* PIP_SHM_H_INCLUDED */
