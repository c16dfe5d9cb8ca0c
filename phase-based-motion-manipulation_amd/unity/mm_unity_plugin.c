/*
 * mm_unity_plugin.c — Unity native rendering-plugin shim around include/mm.h
 * (SURVEY.md §8f row f4): the engine-side half of the zero-copy drop-in for
 *   [RequireComponent(typeof(Camera))] MotionMagnificationProcessor.OnRenderImage
 *   (Assets/Scripts/MotionMagnificationProcessor.cs:4-5, :101-143).
 *
 * UNVERIFIED SKETCH — NOT COMPILED OR RUN IN THIS REPOSITORY: it needs Unity's
 * PluginAPI headers (IUnityInterface.h, IUnityGraphics.h, IUnityGraphicsVulkan.h,
 * shipped with the editor under Editor/Data/PluginAPI) and the Vulkan SDK
 * headers, neither of which is in this image, and a Unity player to run in.
 * Build it next to a Unity project with
 *   cc -O2 -fPIC -shared -I<Unity>/Editor/Data/PluginAPI -I<VulkanSDK>/include \
 *      -Iinclude mm_unity_plugin.c -Llib -lmm355 -lvulkan -o Assets/Plugins/x86_64/libmm355_unity.so
 * What it calls on the HIP side (mm_import_frames, mm_process with
 * MM_FRAMES_ON_DEVICE) is built and tested here (tests/test_extmem.py).
 *
 * Per frame, ONE render-thread event (C# OnRenderImage(source, destination)
 * issues cmd.IssuePluginEventAndData(mm_unity_event_func(),
 * MM_UNITY_EVENT_PROCESS, frame)), configured at load so that Unity submits
 * the command buffers it has recorded so far (source is rendered) and lets
 * the plugin submit on the graphics queue itself (ConfigureEvent:
 * FlushCommandBuffers, queue access Allow, outside a render pass).  One
 * timeline semaphore shared with HIP orders the three legs of frame i:
 *
 *   X_i  (plugin Vulkan submit)  waits 3i   : copy source -> buf[0]     signals 3i+1
 *   H_i  (HIP, the handle's stream) waits 3i+1: mm_process(buf[0] -> buf[1]) signals 3i+2
 *   Y_i  (plugin Vulkan submit)  waits 3i+2 : copy buf[1] -> destination signals 3i+3
 *
 * so X_{i+1} starts only after Y_i has read buf[1] and H_i has read buf[0],
 * and destination receives frame i's OWN output within frame i's event (no
 * one-frame lag).  Frame 0 passes through bitwise inside mm_process
 * (.cs:111-117), so destination = source on the first frame too.  If
 * mm_process fails, H_i copies buf[0] to buf[1] instead (the passthrough
 * Blit of .cs:103-107) and the chain still advances.
 * The texture layouts are read with AccessTexture(..., ObserveOnly), moved to
 * TRANSFER_SRC/DST for the copies and restored, inside the plugin's own
 * command buffers (two sets, re-recorded after a host wait for the value the
 * set's previous use signalled).
 */
#include <stdint.h>
#include <string.h>

#include <vulkan/vulkan.h>
#include <hip/hip_runtime_api.h>

#include "IUnityGraphics.h"
#include "IUnityGraphicsVulkan.h"
#include "IUnityInterface.h"
#include "mm.h"

enum { MM_UNITY_EVENT_PROCESS = 1 };

/* What C# passes with IssuePluginEventAndData (pinned, one per camera). */
typedef struct mm_unity_frame {
    mm_handle *h;           /* from mm_unity_create */
    void *source;           /* RenderTexture.GetNativeTexturePtr() */
    void *destination;
    int width, height;      /* Screen.width / height at Start (.cs:298-302) */
} mm_unity_frame;

/* Interop state of one handle: exportable buffers + semaphore, imported once. */
typedef struct interop {
    mm_handle *h;
    VkDevice dev;
    VkQueue queue;
    VkBuffer buf[2];                 /* 0: input frame, 1: output frame (tightly packed texels,
                                        sized for the widest format, 16 B/px) */
    VkDeviceMemory mem[2];
    mm_ext_frames *ext[2];           /* the same memory as HIP device pointers */
    size_t frame_bytes;
    VkSemaphore sem;                 /* timeline, values 3i .. 3i+3 for frame i */
    hipExternalSemaphore_t hsem;
    uint64_t frame;                  /* frames submitted */
    VkCommandPool pool;
    VkCommandBuffer cb[2][2];        /* [set = frame & 1][0: copy in, 1: copy out] */
    uint64_t set_done[2];            /* timeline value that ends the set's last use */
    hipStream_t stream;
    PFN_vkWaitSemaphores wait_sem;
    PFN_vkSignalSemaphore signal_sem;
    int broken;                      /* a leg failed: later events return at once and
                                        mm_unity_event_ok() tells C# to Blit instead */
} interop;

/* Host waits on the timeline are bounded: a chain that cannot complete (a
 * device lost, a failed leg the repair below could not close) must not hang
 * Unity's render thread.  A timeout is retried (a slow frame is not a lost
 * device) up to MM_UNITY_WAIT_TRIES times before the interop gives up. */
#define MM_UNITY_WAIT_NS 2000000000ull
#define MM_UNITY_WAIT_TRIES 5

static IUnityInterfaces *s_unity;
static IUnityGraphics *s_graphics;
static IUnityGraphicsVulkan *s_vulkan;
static interop s_io;                 /* one camera (the reference has one component) */

static uint32_t memory_type(VkPhysicalDevice pd, uint32_t bits, VkMemoryPropertyFlags want)
{
    VkPhysicalDeviceMemoryProperties mp;
    vkGetPhysicalDeviceMemoryProperties(pd, &mp);
    for (uint32_t i = 0; i < mp.memoryTypeCount; ++i)
        if ((bits & (1u << i)) && (mp.memoryTypes[i].propertyFlags & want) == want) return i;
    return UINT32_MAX;
}

/* One exportable device-local buffer, exported as an opaque fd and imported
 * into the handle's HIP device (mm_import_frames owns the fd afterwards). */
static int make_shared_buffer(const UnityVulkanInstance *vi, size_t bytes, int k)
{
    VkExternalMemoryBufferCreateInfo ext = {VK_STRUCTURE_TYPE_EXTERNAL_MEMORY_BUFFER_CREATE_INFO, NULL,
                                            VK_EXTERNAL_MEMORY_HANDLE_TYPE_OPAQUE_FD_BIT};
    VkBufferCreateInfo bi = {VK_STRUCTURE_TYPE_BUFFER_CREATE_INFO, &ext, 0, bytes,
                             VK_BUFFER_USAGE_TRANSFER_SRC_BIT | VK_BUFFER_USAGE_TRANSFER_DST_BIT,
                             VK_SHARING_MODE_EXCLUSIVE, 0, NULL};
    if (vkCreateBuffer(vi->device, &bi, NULL, &s_io.buf[k]) != VK_SUCCESS) return MM_ERR_HIP;
    VkMemoryRequirements req;
    vkGetBufferMemoryRequirements(vi->device, s_io.buf[k], &req);
    const uint32_t mt = memory_type(vi->physicalDevice, req.memoryTypeBits, VK_MEMORY_PROPERTY_DEVICE_LOCAL_BIT);
    if (mt == UINT32_MAX) return MM_ERR_UNSUPPORTED;
    VkExportMemoryAllocateInfo ex = {VK_STRUCTURE_TYPE_EXPORT_MEMORY_ALLOCATE_INFO, NULL,
                                     VK_EXTERNAL_MEMORY_HANDLE_TYPE_OPAQUE_FD_BIT};
    VkMemoryAllocateInfo ai = {VK_STRUCTURE_TYPE_MEMORY_ALLOCATE_INFO, &ex, req.size, mt};
    if (vkAllocateMemory(vi->device, &ai, NULL, &s_io.mem[k]) != VK_SUCCESS) return MM_ERR_OOM;
    if (vkBindBufferMemory(vi->device, s_io.buf[k], s_io.mem[k], 0) != VK_SUCCESS) return MM_ERR_HIP;
    VkMemoryGetFdInfoKHR gi = {VK_STRUCTURE_TYPE_MEMORY_GET_FD_INFO_KHR, NULL, s_io.mem[k],
                               VK_EXTERNAL_MEMORY_HANDLE_TYPE_OPAQUE_FD_BIT};
    int fd = -1;
    PFN_vkGetMemoryFdKHR get_fd = (PFN_vkGetMemoryFdKHR)vkGetDeviceProcAddr(vi->device, "vkGetMemoryFdKHR");
    if (!get_fd || get_fd(vi->device, &gi, &fd) != VK_SUCCESS) return MM_ERR_HIP;
    return mm_import_frames(s_io.h, fd, req.size, 0, &s_io.ext[k]);   /* include/mm.h, ABI 6 */
}

/* Timeline semaphore (initial value 0) shared with HIP. */
static int make_shared_semaphore(const UnityVulkanInstance *vi)
{
    VkSemaphoreTypeCreateInfo ti = {VK_STRUCTURE_TYPE_SEMAPHORE_TYPE_CREATE_INFO, NULL,
                                    VK_SEMAPHORE_TYPE_TIMELINE, 0};
    VkExportSemaphoreCreateInfo ex = {VK_STRUCTURE_TYPE_EXPORT_SEMAPHORE_CREATE_INFO, &ti,
                                      VK_EXTERNAL_SEMAPHORE_HANDLE_TYPE_OPAQUE_FD_BIT};
    VkSemaphoreCreateInfo si = {VK_STRUCTURE_TYPE_SEMAPHORE_CREATE_INFO, &ex, 0};
    if (vkCreateSemaphore(vi->device, &si, NULL, &s_io.sem) != VK_SUCCESS) return MM_ERR_HIP;
    VkSemaphoreGetFdInfoKHR gi = {VK_STRUCTURE_TYPE_SEMAPHORE_GET_FD_INFO_KHR, NULL, s_io.sem,
                                  VK_EXTERNAL_SEMAPHORE_HANDLE_TYPE_OPAQUE_FD_BIT};
    int fd = -1;
    PFN_vkGetSemaphoreFdKHR get_fd =
        (PFN_vkGetSemaphoreFdKHR)vkGetDeviceProcAddr(vi->device, "vkGetSemaphoreFdKHR");
    if (!get_fd || get_fd(vi->device, &gi, &fd) != VK_SUCCESS) return MM_ERR_HIP;
    hipExternalSemaphoreHandleDesc hd;
    memset(&hd, 0, sizeof hd);
    hd.type = hipExternalSemaphoreHandleTypeTimelineSemaphoreFd;
    hd.handle.fd = fd;
    if (hipImportExternalSemaphore(&s_io.hsem, &hd) != hipSuccess) return MM_ERR_HIP;
    s_io.wait_sem = (PFN_vkWaitSemaphores)vkGetDeviceProcAddr(vi->device, "vkWaitSemaphores");
    s_io.signal_sem = (PFN_vkSignalSemaphore)vkGetDeviceProcAddr(vi->device, "vkSignalSemaphore");
    return s_io.wait_sem && s_io.signal_sem ? MM_OK : MM_ERR_UNSUPPORTED;
}

static int make_command_buffers(const UnityVulkanInstance *vi)
{
    VkCommandPoolCreateInfo pi = {VK_STRUCTURE_TYPE_COMMAND_POOL_CREATE_INFO, NULL,
                                  VK_COMMAND_POOL_CREATE_RESET_COMMAND_BUFFER_BIT, vi->queueFamilyIndex};
    if (vkCreateCommandPool(vi->device, &pi, NULL, &s_io.pool) != VK_SUCCESS) return MM_ERR_HIP;
    VkCommandBufferAllocateInfo ai = {VK_STRUCTURE_TYPE_COMMAND_BUFFER_ALLOCATE_INFO, NULL, s_io.pool,
                                      VK_COMMAND_BUFFER_LEVEL_PRIMARY, 4};
    return vkAllocateCommandBuffers(vi->device, &ai, &s_io.cb[0][0]) == VK_SUCCESS ? MM_OK : MM_ERR_HIP;
}

/* ---- exported to C# (DllImport "mm355_unity") -------------------------- */

UNITY_INTERFACE_EXPORT void UNITY_INTERFACE_API mm_unity_destroy(mm_handle *h);

/* Start / InitializeProcessor (.cs:90-94).  Vulkan renderer only; on any
 * failure everything built so far is released and *out is NULL (C# then
 * keeps the passthrough Blit, .cs:103-107). */
UNITY_INTERFACE_EXPORT int UNITY_INTERFACE_API mm_unity_create(int width, int height, const mm_params *p,
                                                               mm_handle **out)
{
    if (!out) return MM_ERR_INVALID;
    *out = NULL;
    if (!s_vulkan) return MM_ERR_UNSUPPORTED;   /* not the Vulkan renderer (UnityPluginLoad) */
    if (s_io.h) return MM_ERR_INVALID;          /* one camera per plugin instance */
    int rc = mm_create(width, height, p, 0, &s_io.h);
    if (rc) {
        memset(&s_io, 0, sizeof s_io);
        return rc;
    }
    const UnityVulkanInstance vi = s_vulkan->Instance();
    s_io.dev = vi.device;
    s_io.queue = vi.graphicsQueue;
    s_io.stream = (hipStream_t)mm_stream(s_io.h);
    s_io.frame_bytes = (size_t)width * height * 16;   /* any format (unity_frame_format) fits */
    if ((rc = make_shared_buffer(&vi, s_io.frame_bytes, 0)) || (rc = make_shared_buffer(&vi, s_io.frame_bytes, 1)) ||
        (rc = make_shared_semaphore(&vi)) || (rc = make_command_buffers(&vi))) {
        mm_unity_destroy(s_io.h);
        return rc;
    }
    *out = s_io.h;
    return MM_OK;
}

/* Image barrier inside the plugin's own command buffer. */
static void transition(VkCommandBuffer cb, VkImage img, VkImageLayout from, VkImageLayout to,
                       VkAccessFlags src_access, VkAccessFlags dst_access)
{
    VkImageMemoryBarrier b;
    memset(&b, 0, sizeof b);
    b.sType = VK_STRUCTURE_TYPE_IMAGE_MEMORY_BARRIER;
    b.srcAccessMask = src_access;
    b.dstAccessMask = dst_access;
    b.oldLayout = from;
    b.newLayout = to;
    b.srcQueueFamilyIndex = VK_QUEUE_FAMILY_IGNORED;
    b.dstQueueFamilyIndex = VK_QUEUE_FAMILY_IGNORED;
    b.image = img;
    b.subresourceRange.aspectMask = VK_IMAGE_ASPECT_COLOR_BIT;
    b.subresourceRange.levelCount = 1;
    b.subresourceRange.layerCount = 1;
    vkCmdPipelineBarrier(cb, VK_PIPELINE_STAGE_ALL_COMMANDS_BIT, VK_PIPELINE_STAGE_ALL_COMMANDS_BIT, 0, 0, NULL, 0,
                         NULL, 1, &b);
}

/* Records the copy between one texture and one interop buffer (to_buffer:
 * image -> buffer, else buffer -> image), the texture left in its layout. */
static int record_copy(VkCommandBuffer cb, const UnityVulkanImage *img, VkBuffer buf, int to_buffer,
                       int width, int height)
{
    if (vkResetCommandBuffer(cb, 0) != VK_SUCCESS) return 0;
    VkCommandBufferBeginInfo bi = {VK_STRUCTURE_TYPE_COMMAND_BUFFER_BEGIN_INFO, NULL,
                                   VK_COMMAND_BUFFER_USAGE_ONE_TIME_SUBMIT_BIT, NULL};
    if (vkBeginCommandBuffer(cb, &bi) != VK_SUCCESS) return 0;
    const VkImageLayout xfer = to_buffer ? VK_IMAGE_LAYOUT_TRANSFER_SRC_OPTIMAL : VK_IMAGE_LAYOUT_TRANSFER_DST_OPTIMAL;
    const VkAccessFlags acc = to_buffer ? VK_ACCESS_TRANSFER_READ_BIT : VK_ACCESS_TRANSFER_WRITE_BIT;
    transition(cb, img->image, img->layout, xfer, VK_ACCESS_MEMORY_WRITE_BIT, acc);
    VkBufferImageCopy rg;
    memset(&rg, 0, sizeof rg);
    rg.imageSubresource.aspectMask = VK_IMAGE_ASPECT_COLOR_BIT;
    rg.imageSubresource.layerCount = 1;
    rg.imageExtent.width = (uint32_t)width;
    rg.imageExtent.height = (uint32_t)height;
    rg.imageExtent.depth = 1;
    if (to_buffer) vkCmdCopyImageToBuffer(cb, img->image, xfer, buf, 1, &rg);
    else vkCmdCopyBufferToImage(cb, buf, img->image, xfer, 1, &rg);
    transition(cb, img->image, xfer, img->layout, acc, VK_ACCESS_MEMORY_READ_BIT | VK_ACCESS_MEMORY_WRITE_BIT);
    return vkEndCommandBuffer(cb) == VK_SUCCESS;
}

/* One submission of cb that waits for timeline value `wait` and signals `signal`. */
static int submit(VkCommandBuffer cb, uint64_t wait, uint64_t signal)
{
    VkTimelineSemaphoreSubmitInfo ts = {VK_STRUCTURE_TYPE_TIMELINE_SEMAPHORE_SUBMIT_INFO, NULL, 1, &wait, 1, &signal};
    const VkPipelineStageFlags stage = VK_PIPELINE_STAGE_TRANSFER_BIT;
    VkSubmitInfo si = {VK_STRUCTURE_TYPE_SUBMIT_INFO, &ts, 1, &s_io.sem, &stage, 1, &cb, 1, &s_io.sem};
    return vkQueueSubmit(s_io.queue, 1, &si, VK_NULL_HANDLE) == VK_SUCCESS;
}

/* VK_SUCCESS, VK_TIMEOUT after MM_UNITY_WAIT_TRIES bounded waits, or the
 * error (VK_ERROR_DEVICE_LOST) */
static VkResult host_wait_result(uint64_t value)
{
    VkSemaphoreWaitInfo wi = {VK_STRUCTURE_TYPE_SEMAPHORE_WAIT_INFO, NULL, 0, 1, &s_io.sem, &value};
    VkResult r = VK_TIMEOUT;
    for (int k = 0; k < MM_UNITY_WAIT_TRIES && r == VK_TIMEOUT; ++k) r = s_io.wait_sem(s_io.dev, &wi, MM_UNITY_WAIT_NS);
    return r;
}

static int host_wait(uint64_t value) { return host_wait_result(value) == VK_SUCCESS; }

/* include/mm.h frame format of a render target's texels (the reference
 * camera's HDR target is R16G16B16A16_SFLOAT, an LDR one R8G8B8A8_SRGB under
 * Linear colour space); -1: not one the operator takes (BGRA orders
 * included), so the event falls back to the passthrough Blit. */
static int unity_frame_format(VkFormat f)
{
    switch (f) {
    case VK_FORMAT_R8G8B8A8_UNORM: return MM_RGBA8;
    case VK_FORMAT_R8G8B8A8_SRGB: return MM_RGBA8_SRGB;
    case VK_FORMAT_R16G16B16A16_SFLOAT: return MM_RGBA16F;
    case VK_FORMAT_R32G32B32A32_SFLOAT: return MM_RGBA32F;
    default: return -1;
    }
}

static int host_signal(uint64_t value)
{
    VkSemaphoreSignalInfo si = {VK_STRUCTURE_TYPE_SEMAPHORE_SIGNAL_INFO, NULL, s_io.sem, value};
    return s_io.signal_sem(s_io.dev, &si) == VK_SUCCESS;
}

/* A leg of frame i failed after X_i was submitted: bring the timeline to 3i+3
 * from the host (after the legs that did queue have completed, since a
 * timeline value only moves forward), so that nothing queued later waits
 * forever, and stop using the interop (C# falls back to Graphics.Blit). */
static void close_chain(uint64_t reached, uint64_t base)
{
    s_io.broken = 1;
    if (reached > base && !host_wait(reached)) return;   /* device lost: nothing to close */
    if (reached < base + 3) (void)host_signal(base + 3);
    s_io.set_done[0] = s_io.set_done[1] = 0;
}

/* Render-thread callback: the three legs of the header comment. */
static void UNITY_INTERFACE_API on_render_event(int event_id, void *data)
{
    if (event_id != MM_UNITY_EVENT_PROCESS || !s_vulkan || !data || !s_io.h || s_io.broken) return;
    const mm_unity_frame *f = (const mm_unity_frame *)data;
    /* current layouts, no barrier from Unity (the plugin's own command
     * buffers move and restore them) */
    VkImageSubresource sub = {VK_IMAGE_ASPECT_COLOR_BIT, 0, 0};
    UnityVulkanImage src, dst;
    if (!s_vulkan->AccessTexture(f->source, &sub, VK_IMAGE_LAYOUT_UNDEFINED, 0, 0,
                                 kUnityVulkanResourceAccess_ObserveOnly, &src) ||
        !s_vulkan->AccessTexture(f->destination, &sub, VK_IMAGE_LAYOUT_UNDEFINED, 0, 0,
                                 kUnityVulkanResourceAccess_ObserveOnly, &dst))
        return;
    /* source and destination share the camera's format (Blit(source,
     * destination) of the reference keeps it); the interop buffers hold any */
    const int fmt = unity_frame_format(src.format);
    if (fmt < 0 || unity_frame_format(dst.format) != fmt) {
        s_io.broken = 1;   /* C# Blits (mm_unity_event_ok) */
        return;
    }
    const uint64_t i = s_io.frame, base = 3 * i;
    const int set = (int)(i & 1);
    /* the set's command buffers were last submitted for frame i-2 */
    if (s_io.set_done[set] && !host_wait(s_io.set_done[set])) {
        s_io.broken = 1;
        return;
    }
    if (!record_copy(s_io.cb[set][0], &src, s_io.buf[0], 1, f->width, f->height) ||
        !record_copy(s_io.cb[set][1], &dst, s_io.buf[1], 0, f->width, f->height))
        return;   /* nothing submitted: the timeline stays at 3i */
    /* X_i: source -> buf[0] after Y_{i-1} (value 3i) */
    if (!submit(s_io.cb[set][0], base, base + 1)) return;
    s_io.frame = i + 1;   /* from here on the chain must reach 3i+3 */
    /* H_i: mm_process on the imported buffers, between 3i+1 and 3i+2.  If the
     * stream cannot be made to wait for X_i, waiting on the host for it keeps
     * mm_process from reading buf[0] early. */
    hipExternalSemaphoreWaitParams wp;
    memset(&wp, 0, sizeof wp);
    wp.params.fence.value = base + 1;
    if (hipWaitExternalSemaphoresAsync(&s_io.hsem, &wp, 1, s_io.stream) != hipSuccess && !host_wait(base + 1)) {
        close_chain(base + 1, base);
        return;
    }
    void *in = mm_ext_frames_ptr(s_io.ext[0]), *out = mm_ext_frames_ptr(s_io.ext[1]);
    size_t fb = 0;
    (void)mm_frame_bytes(f->width, f->height, fmt, &fb);
    if (mm_process(f->h, in, out, fmt, MM_FRAMES_ON_DEVICE, s_io.stream) != MM_OK &&
        hipMemcpyAsync(out, in, fb, hipMemcpyDeviceToDevice, s_io.stream) != hipSuccess) {   /* .cs:105 */
        (void)hipStreamSynchronize(s_io.stream);
        close_chain(base + 1, base);
        return;
    }
    hipExternalSemaphoreSignalParams sp;
    memset(&sp, 0, sizeof sp);
    sp.params.fence.value = base + 2;
    if (hipSignalExternalSemaphoresAsync(&s_io.hsem, &sp, 1, s_io.stream) != hipSuccess) {
        /* H_i's work is queued but will not signal: finish it on the host */
        (void)hipStreamSynchronize(s_io.stream);
        close_chain(base + 1, base);
        return;
    }
    /* Y_i: buf[1] -> destination after H_i, in this same event */
    if (!submit(s_io.cb[set][1], base + 2, base + 3)) {
        close_chain(base + 2, base);
        return;
    }
    s_io.set_done[set] = base + 3;
}

/* For C#: false once the interop has failed (then OnRenderImage Blits source
 * to destination itself, the reference's error path .cs:103-107). */
UNITY_INTERFACE_EXPORT int UNITY_INTERFACE_API mm_unity_event_ok(void)
{
    return s_io.h && !s_io.broken;
}

UNITY_INTERFACE_EXPORT UnityRenderingEventAndData UNITY_INTERFACE_API mm_unity_event_func(void)
{
    return on_render_event;
}

/* OnDestroy -> ReleaseResources (.cs:96-99): waits for the last frame's chain,
 * then releases in reverse order of creation (safe on a partial create).  The
 * Vulkan objects are freed only once the chain is known to be done (the wait
 * returned VK_SUCCESS) or can never run again (VK_ERROR_DEVICE_LOST); if it
 * is still pending after the retried waits, a queued copy may still use the
 * buffers, their memory and the semaphore, so they are leaked instead. */
UNITY_INTERFACE_EXPORT void UNITY_INTERFACE_API mm_unity_destroy(mm_handle *h)
{
    if (!h || h != s_io.h) return;
    int vk_free = 1;
    if (s_io.frame && s_io.wait_sem) {
        const VkResult r = host_wait_result(3 * s_io.frame);
        vk_free = r == VK_SUCCESS || r == VK_ERROR_DEVICE_LOST;
    }
    if (s_io.stream) (void)hipStreamSynchronize(s_io.stream);
    for (int k = 0; k < 2; ++k)
        if (s_io.ext[k]) mm_release_frames(s_io.ext[k]);
    if (s_io.hsem) (void)hipDestroyExternalSemaphore(s_io.hsem);
    mm_destroy(h);
    if (s_io.dev && vk_free) {
        if (s_io.pool) vkDestroyCommandPool(s_io.dev, s_io.pool, NULL);   /* frees the command buffers */
        for (int k = 0; k < 2; ++k) {
            if (s_io.buf[k]) vkDestroyBuffer(s_io.dev, s_io.buf[k], NULL);
            if (s_io.mem[k]) vkFreeMemory(s_io.dev, s_io.mem[k], NULL);
        }
        if (s_io.sem) vkDestroySemaphore(s_io.dev, s_io.sem, NULL);
    }
    memset(&s_io, 0, sizeof s_io);
}

/* ---- Unity plugin entry points ----------------------------------------- */

UNITY_INTERFACE_EXPORT void UNITY_INTERFACE_API UnityPluginLoad(IUnityInterfaces *unity)
{
    s_unity = unity;
    s_graphics = UNITY_GET_INTERFACE(unity, IUnityGraphics);
    s_vulkan = UNITY_GET_INTERFACE(unity, IUnityGraphicsVulkan);   /* NULL on other renderers */
    if (s_vulkan) {
        /* the event submits on the graphics queue itself: Unity first submits
         * what it has recorded (the rendered source), outside a render pass */
        UnityVulkanPluginEventConfig cfg;
        memset(&cfg, 0, sizeof cfg);
        cfg.renderPassPrecondition = kUnityVulkanRenderPass_EnsureOutside;
        cfg.graphicsQueueAccess = kUnityVulkanGraphicsQueueAccess_Allow;
        cfg.flags = kUnityVulkanEventConfigFlag_EnsurePreviousFrameSubmission |
                    kUnityVulkanEventConfigFlag_FlushCommandBuffers | kUnityVulkanEventConfigFlag_SyncWorkerThreads;
        s_vulkan->ConfigureEvent(MM_UNITY_EVENT_PROCESS, &cfg);
    }
}

UNITY_INTERFACE_EXPORT void UNITY_INTERFACE_API UnityPluginUnload(void)
{
    s_vulkan = NULL;
    s_graphics = NULL;
    s_unity = NULL;
}
