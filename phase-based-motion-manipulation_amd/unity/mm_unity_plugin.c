/*
 * mm_unity_plugin.c — Unity native rendering-plugin shim around include/mm.h
 * (SURVEY.md §8f row f4): the engine-side half of the zero-copy drop-in for
 *   [RequireComponent(typeof(Camera))] MotionMagnificationProcessor.OnRenderImage
 *   (Assets/Scripts/MotionMagnificationProcessor.cs:4-5, :101-143).
 *
 * NOT COMPILED IN THIS REPOSITORY: it needs Unity's PluginAPI headers
 * (IUnityInterface.h, IUnityGraphics.h, IUnityGraphicsVulkan.h, shipped with the
 * editor under Editor/Data/PluginAPI) and the Vulkan SDK headers, neither of
 * which is in this image.  Build it next to a Unity project with
 *   cc -O2 -fPIC -shared -I<Unity>/Editor/Data/PluginAPI -I<VulkanSDK>/include \
 *      -Iinclude mm_unity_plugin.c -Llib -lmm355 -o Assets/Plugins/x86_64/libmm355_unity.so
 * What it calls on the HIP side (mm_import_frames, mm_process with
 * MM_FRAMES_ON_DEVICE) is built and tested here (tests/test_extmem.py).
 *
 * Data path per frame (render thread, Vulkan renderer):
 *   1. C# OnRenderImage(source, destination) records
 *        cmd.IssuePluginEventAndData(mm_unity_event_func(), MM_UNITY_EVENT_PROCESS, frame)
 *      with `frame` -> struct mm_unity_frame {handle, source, destination textures}.
 *   2. Here, inside Unity's command recording (IUnityGraphicsVulkan::
 *      CommandRecordingState): copy `source` into an exportable linear buffer
 *      (vkCmdCopyImageToBuffer; the RenderTexture's own memory is not
 *      allocated exportable), signal an exportable timeline semaphore.
 *   3. HIP side: the buffers were exported once (vkGetMemoryFdKHR) and imported
 *      once (mm_import_frames); the semaphore likewise (hipImportExternalSemaphore).
 *      hipWaitExternalSemaphoresAsync -> mm_process(in, out, MM_RGBA8,
 *      MM_FRAMES_ON_DEVICE, stream) -> hipSignalExternalSemaphoresAsync.
 *   4. Next recording: wait on that semaphore value and copy the output buffer
 *      into `destination` (vkCmdCopyBufferToImage).
 * The first frame after Start passes through bitwise (.cs:111-117) inside
 * mm_process itself; errors fall back to Graphics.Blit on the C# side
 * (.cs:103-107) because every mm_* call returns a code.
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
    VkBuffer buf[2];                 /* 0: input frame, 1: output frame (linear RGBA8) */
    VkDeviceMemory mem[2];
    mm_ext_frames *ext[2];           /* the same memory as HIP device pointers */
    VkSemaphore sem;                 /* timeline: Vulkan copy-in done / HIP done */
    hipExternalSemaphore_t hsem;
    uint64_t value;
    hipStream_t stream;
} interop;

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
    VkExportMemoryAllocateInfo ex = {VK_STRUCTURE_TYPE_EXPORT_MEMORY_ALLOCATE_INFO, NULL,
                                     VK_EXTERNAL_MEMORY_HANDLE_TYPE_OPAQUE_FD_BIT};
    VkMemoryAllocateInfo ai = {VK_STRUCTURE_TYPE_MEMORY_ALLOCATE_INFO, &ex, req.size,
                               memory_type(vi->physicalDevice, req.memoryTypeBits,
                                           VK_MEMORY_PROPERTY_DEVICE_LOCAL_BIT)};
    if (vkAllocateMemory(vi->device, &ai, NULL, &s_io.mem[k]) != VK_SUCCESS ||
        vkBindBufferMemory(vi->device, s_io.buf[k], s_io.mem[k], 0) != VK_SUCCESS)
        return MM_ERR_OOM;
    VkMemoryGetFdInfoKHR gi = {VK_STRUCTURE_TYPE_MEMORY_GET_FD_INFO_KHR, NULL, s_io.mem[k],
                               VK_EXTERNAL_MEMORY_HANDLE_TYPE_OPAQUE_FD_BIT};
    int fd = -1;
    PFN_vkGetMemoryFdKHR get_fd = (PFN_vkGetMemoryFdKHR)vkGetDeviceProcAddr(vi->device, "vkGetMemoryFdKHR");
    if (!get_fd || get_fd(vi->device, &gi, &fd) != VK_SUCCESS) return MM_ERR_HIP;
    return mm_import_frames(s_io.h, fd, req.size, 0, &s_io.ext[k]);   /* include/mm.h, ABI 6 */
}

/* Timeline semaphore shared with HIP: Vulkan signals odd values (input copied),
 * HIP signals even values (output written). */
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
    return MM_OK;
}

/* ---- exported to C# (DllImport "mm355_unity") -------------------------- */

UNITY_INTERFACE_EXPORT int UNITY_INTERFACE_API mm_unity_create(int width, int height, const mm_params *p,
                                                               mm_handle **out)
{
    int rc = mm_create(width, height, p, 0, out);   /* Start / InitializeProcessor (.cs:90-94) */
    if (rc) return rc;
    s_io.h = *out;
    s_io.stream = (hipStream_t)mm_stream(*out);
    const UnityVulkanInstance vi = s_vulkan->Instance();
    const size_t bytes = (size_t)width * height * 4;
    if ((rc = make_shared_buffer(&vi, bytes, 0)) || (rc = make_shared_buffer(&vi, bytes, 1)) ||
        (rc = make_shared_semaphore(&vi)))
        return rc;
    return MM_OK;
}

/* Render-thread callback: steps 2-4 of the header comment. */
static void UNITY_INTERFACE_API on_render_event(int event_id, void *data)
{
    if (event_id != MM_UNITY_EVENT_PROCESS || !s_vulkan || !data) return;
    const mm_unity_frame *f = (const mm_unity_frame *)data;
    UnityVulkanRecordingState rs;
    if (!s_vulkan->CommandRecordingState(&rs, kUnityVulkanGraphicsQueueAccess_DontCare)) return;
    VkImageSubresource sub = {VK_IMAGE_ASPECT_COLOR_BIT, 0, 0};
    UnityVulkanImage src, dst;
    if (!s_vulkan->AccessTexture(f->source, &sub, VK_IMAGE_LAYOUT_TRANSFER_SRC_OPTIMAL,
                                 VK_PIPELINE_STAGE_TRANSFER_BIT, VK_ACCESS_TRANSFER_READ_BIT,
                                 kUnityVulkanResourceAccess_PipelineBarrier, &src) ||
        !s_vulkan->AccessTexture(f->destination, &sub, VK_IMAGE_LAYOUT_TRANSFER_DST_OPTIMAL,
                                 VK_PIPELINE_STAGE_TRANSFER_BIT, VK_ACCESS_TRANSFER_WRITE_BIT,
                                 kUnityVulkanResourceAccess_PipelineBarrier, &dst))
        return;
    VkBufferImageCopy rg;
    memset(&rg, 0, sizeof rg);
    rg.imageSubresource.aspectMask = VK_IMAGE_ASPECT_COLOR_BIT;
    rg.imageSubresource.layerCount = 1;
    rg.imageExtent.width = (uint32_t)f->width;
    rg.imageExtent.height = (uint32_t)f->height;
    rg.imageExtent.depth = 1;
    /* the previous frame's output (HIP signalled value) lands in destination */
    if (s_io.value) vkCmdCopyBufferToImage(rs.commandBuffer, s_io.buf[1], dst.image,
                                           VK_IMAGE_LAYOUT_TRANSFER_DST_OPTIMAL, 1, &rg);
    vkCmdCopyImageToBuffer(rs.commandBuffer, src.image, VK_IMAGE_LAYOUT_TRANSFER_SRC_OPTIMAL,
                           s_io.buf[0], 1, &rg);
    /* Unity submits rs.commandBuffer; its end-of-frame submit signals
     * s_io.sem = value+1 (registered through IUnityGraphicsVulkan's
     * ConfigureEvent / the frame's signal semaphore list). */
    const uint64_t copied = ++s_io.value;
    hipExternalSemaphoreWaitParams wp;
    memset(&wp, 0, sizeof wp);
    wp.params.fence.value = copied;
    if (hipWaitExternalSemaphoresAsync(&s_io.hsem, &wp, 1, s_io.stream) != hipSuccess) return;
    if (mm_process(f->h, mm_ext_frames_ptr(s_io.ext[0]), mm_ext_frames_ptr(s_io.ext[1]), MM_RGBA8,
                   MM_FRAMES_ON_DEVICE, s_io.stream) != MM_OK)
        return;   /* C# sees no new output and keeps blitting (.cs:103-107) */
    hipExternalSemaphoreSignalParams sp;
    memset(&sp, 0, sizeof sp);
    sp.params.fence.value = ++s_io.value;
    (void)hipSignalExternalSemaphoresAsync(&s_io.hsem, &sp, 1, s_io.stream);
}

UNITY_INTERFACE_EXPORT UnityRenderingEventAndData UNITY_INTERFACE_API mm_unity_event_func(void)
{
    return on_render_event;
}

UNITY_INTERFACE_EXPORT void UNITY_INTERFACE_API mm_unity_destroy(mm_handle *h)
{
    for (int k = 0; k < 2; ++k)
        if (s_io.ext[k]) mm_release_frames(s_io.ext[k]);
    if (s_io.hsem) (void)hipDestroyExternalSemaphore(s_io.hsem);
    mm_destroy(h);                                   /* OnDestroy -> ReleaseResources (.cs:96-99) */
    if (s_vulkan) {
        const UnityVulkanInstance vi = s_vulkan->Instance();
        for (int k = 0; k < 2; ++k) {
            vkDestroyBuffer(vi.device, s_io.buf[k], NULL);
            vkFreeMemory(vi.device, s_io.mem[k], NULL);
        }
        vkDestroySemaphore(vi.device, s_io.sem, NULL);
    }
    memset(&s_io, 0, sizeof s_io);
}

/* ---- Unity plugin entry points ----------------------------------------- */

UNITY_INTERFACE_EXPORT void UNITY_INTERFACE_API UnityPluginLoad(IUnityInterfaces *unity)
{
    s_unity = unity;
    s_graphics = UNITY_GET_INTERFACE(unity, IUnityGraphics);
    s_vulkan = UNITY_GET_INTERFACE(unity, IUnityGraphicsVulkan);   /* NULL on other renderers */
}

UNITY_INTERFACE_EXPORT void UNITY_INTERFACE_API UnityPluginUnload(void)
{
    s_vulkan = NULL;
    s_graphics = NULL;
    s_unity = NULL;
}
