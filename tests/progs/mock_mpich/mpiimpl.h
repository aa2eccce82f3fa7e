/*
 * mock_mpich/mpiimpl.h -- test stand-in for the few things of MPICH's internal
 * header that csrc/host/mpich_glue.c and the mock libmpi use: the per-thread
 * struct with op_errno and its access macro, and the critical-section macros
 * at each thread granularity.  Written for the tests from the behaviour of
 * src/include/mpir_thread.h:61-82 (MPIR_Per_thread_t, MPIR_Per_thread with a
 * TLS specifier) and src/mpid/common/thread/mpidu_thread_fallback.h:95-170
 * (GLOBAL: one recursive mutex, POBJ / VCI empty; POBJ: GLOBAL empty, POBJ a
 * non-recursive mutex per object class; VCI: GLOBAL and VCI recursive).  Only
 * active when MPIR_ThreadInfo.isThreaded, as in MPICH.
 *
 * MOCK_GRANULARITY: 1 GLOBAL (MPICH's default), 2 POBJ, 3 VCI.
 */
#ifndef MOCK_MPIIMPL_H_INCLUDED
#define MOCK_MPIIMPL_H_INCLUDED

#include <assert.h>
#include <pthread.h>

#ifndef MOCK_GRANULARITY
#define MOCK_GRANULARITY 1
#endif

typedef struct {
    int op_errno;
    char strerrbuf[1024];
    int lock_depth;
} MPIR_Per_thread_t;

extern __thread MPIR_Per_thread_t MPIR_Per_thread;
typedef int MPID_Thread_tls_t;
extern MPID_Thread_tls_t MPIR_Per_thread_key;

typedef struct {
    int isThreaded;
} MPIR_Thread_info_t;
extern MPIR_Thread_info_t MPIR_ThreadInfo;

#define MPIR_Assert(x) assert(x)

/* MPL_THREADPRIV_KEY_GET_ADDR with a TLS specifier: the variable's address */
#define MPID_THREADPRIV_KEY_GET_ADDR(is_threaded, key, var, addr, err_ptr) \
    do { (void) (is_threaded); (void) (key); (addr) = &(var); *(err_ptr) = 0; } while (0)

typedef struct {
    pthread_mutex_t m;
    int recursive;
} MPID_Thread_mutex_t;

extern MPID_Thread_mutex_t MPIR_THREAD_GLOBAL_ALLFUNC_MUTEX;
extern MPID_Thread_mutex_t MPIR_THREAD_POBJ_HANDLE_MUTEX;

/* counts of lock acquisitions, so the tests can see which sections ran */
extern int mock_cs_global_enters, mock_cs_handle_enters;

#define MOCK_LOCK(mx, counter)                                  \
    do { if (MPIR_ThreadInfo.isThreaded) {                      \
            pthread_mutex_lock(&(mx).m);                        \
            __atomic_add_fetch(&(counter), 1, __ATOMIC_RELAXED); \
        } } while (0)
#define MOCK_UNLOCK(mx)                                         \
    do { if (MPIR_ThreadInfo.isThreaded) pthread_mutex_unlock(&(mx).m); } while (0)
#define MOCK_NOTHING(mx) do { (void) 0; } while (0)

#if MOCK_GRANULARITY == 1
#define MOCK_CS_ENTER_GLOBAL(mx) MOCK_LOCK(mx, mock_cs_global_enters)
#define MOCK_CS_EXIT_GLOBAL(mx)  MOCK_UNLOCK(mx)
#define MOCK_CS_ENTER_POBJ(mx)   MOCK_NOTHING(mx)
#define MOCK_CS_EXIT_POBJ(mx)    MOCK_NOTHING(mx)
#define MOCK_CS_ENTER_VCI(mx)    MOCK_NOTHING(mx)
#define MOCK_CS_EXIT_VCI(mx)     MOCK_NOTHING(mx)
#elif MOCK_GRANULARITY == 2
#define MOCK_CS_ENTER_GLOBAL(mx) MOCK_NOTHING(mx)
#define MOCK_CS_EXIT_GLOBAL(mx)  MOCK_NOTHING(mx)
#define MOCK_CS_ENTER_POBJ(mx)   MOCK_LOCK(mx, mock_cs_handle_enters)
#define MOCK_CS_EXIT_POBJ(mx)    MOCK_UNLOCK(mx)
#define MOCK_CS_ENTER_VCI(mx)    MOCK_NOTHING(mx)
#define MOCK_CS_EXIT_VCI(mx)     MOCK_NOTHING(mx)
#else
#define MOCK_CS_ENTER_GLOBAL(mx) MOCK_LOCK(mx, mock_cs_global_enters)
#define MOCK_CS_EXIT_GLOBAL(mx)  MOCK_UNLOCK(mx)
#define MOCK_CS_ENTER_POBJ(mx)   MOCK_NOTHING(mx)
#define MOCK_CS_EXIT_POBJ(mx)    MOCK_NOTHING(mx)
#define MOCK_CS_ENTER_VCI(mx)    MOCK_LOCK(mx, mock_cs_handle_enters)
#define MOCK_CS_EXIT_VCI(mx)     MOCK_UNLOCK(mx)
#endif

/* the communicator fields the glue reads (mpir_comm.h:134,148) and the
 * process struct that holds the world (mpir_process.h:34-38) */
typedef struct MPIR_Comm {
    int local_size;
    struct MPIR_Comm *node_comm;
} MPIR_Comm;

typedef struct {
    MPIR_Comm *comm_world;
} MPIR_Process_t;
extern MPIR_Process_t MPIR_Process;

#define MPID_THREAD_CS_ENTER(name, mutex) MOCK_CS_ENTER_##name(mutex)
#define MPID_THREAD_CS_EXIT(name, mutex)  MOCK_CS_EXIT_##name(mutex)

#endif /* MOCK_MPIIMPL_H_INCLUDED */
